// MI355X configuration keys seen by native code: the C++ mirror of the spark.ray.mi355x.*
// entries of raydp_amd/utils/config.py (tests/test_config.py checks the two agree).
//
// Native code runs in processes without a Spark session (actor workers, trainer ranks), so
// it reads the environment variable each key maps to; the Python side exports those
// variables for workers (config.env_for_workers).
#pragma once
#include <stdlib.h>
#include <string.h>

namespace rx_config {

struct Key {
  const char* key;
  const char* env;
  const char* default_value;
};

constexpr Key kKeys[] = {
    {"spark.ray.mi355x.allreduce", "RAYDP_ALLREDUCE", "auto"},
    {"spark.ray.mi355x.allreduce.timeout_s", "RAYDP_ALLREDUCE_TIMEOUT_S", "30"},
    {"spark.ray.mi355x.allreduce.oneshot_max_mb", "RAYDP_ALLREDUCE_ONESHOT_MAX_MB", "16"},
    {"spark.ray.mi355x.allreduce.twoshot_min_mb", "RAYDP_ALLREDUCE_TWOSHOT_MIN_MB", "1"},
    {"spark.ray.mi355x.ddp.comm_stream", "RAYDP_DDP_COMM_STREAM", "auto"},
    {"spark.ray.mi355x.fused", "RAYDP_FUSED", "auto"},
    {"spark.ray.mi355x.hip_graphs", "RAYDP_TORCH_GRAPHS", "1"},
    {"spark.ray.mi355x.mlp_jit", "RAYDP_MLP_JIT", "1"},
    {"spark.ray.mi355x.mlp_wgrad", "RAYDP_MLP_WGRAD", "opt"},
    {"spark.ray.mi355x.mlp_persistent", "RAYDP_MLP_PERSISTENT", "1"},
    {"spark.ray.mi355x.mlp_persistent.timeout_s", "RAYDP_MLP_PERSISTENT_TIMEOUT_S", "5"},
    {"spark.ray.mi355x.fused_linear", "RAYDP_FUSED_LINEAR", "1"},
    {"spark.ray.mi355x.driver_gc_freeze", "RAYDP_DRIVER_GC_FREEZE", "1"},
    {"spark.ray.mi355x.ddp.bucket_mb", "RAYDP_DDP_BUCKET_MB", "0"},
    {"spark.ray.mi355x.ddp.first_bucket_mb", "RAYDP_DDP_FIRST_BUCKET_MB", "1"},
    {"spark.ray.mi355x.ddp.overlap_bucket_mb", "RAYDP_DDP_OVERLAP_BUCKET_MB", "4"},
    {"spark.ray.mi355x.runtime.port", "RAYDP_RUNTIME_PORT", "-1"},
    {"spark.ray.mi355x.runtime.host", "RAYDP_RUNTIME_HOST", "127.0.0.1"},
    {"spark.ray.mi355x.object_store_bytes", "RAYDP_OBJECT_STORE_BYTES", "0"},
    {"spark.ray.mi355x.trace", "RAYDP_TRACE", ""},
    {"spark.ray.mi355x.roctx", "RAYDP_ROCTX", "0"},
    {"spark.ray.mi355x.opt_xcd_affine", "RAYDP_OPT_XCD_AFFINE", "1"},
    {"spark.ray.mi355x.fused_etl", "RAYDP_FUSED_ETL", "1"},
    {"spark.ray.mi355x.local_exec_bytes", "RAYDP_LOCAL_EXEC_BYTES", "4m"},
    {"spark.ray.mi355x.xg_opt_stride", "RAYDP_XG_OPT_STRIDE", "1"},
    {"spark.ray.mi355x.overlap_conversion", "RAYDP_OVERLAP_CONVERSION", "1"},
    {"spark.ray.mi355x.step_times", "RAYDP_STEP_TIMES", "1"},
    {"spark.ray.mi355x.udf_verify", "RAYDP_UDF_VERIFY", "sampled"},
    {"spark.ray.mi355x.native_executor", "RAYDP_NATIVE_EXECUTOR", "1"},
    {"spark.ray.mi355x.fused_optimizer", "RAYDP_FUSED_OPTIMIZER", "1"},
    {"spark.ray.mi355x.native_batchnorm", "RAYDP_NATIVE_BATCHNORM", "1"},
    {"spark.ray.mi355x.graph_user_model", "RAYDP_GRAPH_USER_MODEL", "1"},
    {"spark.ray.mi355x.graph_hvd_model", "RAYDP_GRAPH_HVD_MODEL", "0"},
    {"spark.ray.mi355x.stream_ingest", "RAYDP_STREAM_INGEST", "1"},
    {"spark.ray.mi355x.train_inprocess", "RAYDP_TRAIN_INPROCESS", "1"},
};

// Value of a key: its environment variable when set and non-empty, else the default.
inline const char* get(const char* key) {
  for (const Key& k : kKeys)
    if (strcmp(k.key, key) == 0) {
      const char* v = getenv(k.env);
      return (v && v[0]) ? v : k.default_value;
    }
  return nullptr;
}

inline long get_int(const char* key, long fallback) {
  const char* v = get(key);
  return (v && v[0]) ? strtol(v, nullptr, 10) : fallback;
}

}  // namespace rx_config
