"""Typed configuration registry: every key the framework reads, with type, default and doc.

Parity: the reference's configuration is SparkConf key/value pairs (``init_spark(configs=…)``,
``spark-defaults.conf``, ``--conf``), with RayDP's own keys declared in
``core/raydp-main/src/main/java/org/apache/spark/raydp/SparkOnRayConfigs.java:5-127`` and read
across ``python/raydp/spark/ray_cluster.py:80-189``, ``ray_cluster_master.py:35-49`` and
``RayCoarseGrainedSchedulerBackend.scala:177-228``. The same key names are
accepted here so user code ports unchanged; keys that only configure the JVM (class paths,
log4j, the java agent) are registered as ``ignored`` and logged at debug level when set.

New MI355X keys live under ``spark.ray.mi355x.*``. Each registered key can also be set by an
environment variable (``env``), which is how settings reach worker processes that have no
Spark session (trainer workers, the bench). Precedence: explicit ``conf`` mapping > active
session conf > environment > default.

The C++ side mirrors the MI355X keys in ``csrc/common/config_keys.h`` (checked by
``tests/test_config.py``).
"""
import logging
import os
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Iterable, List, Mapping, Optional

log = logging.getLogger(__name__)


def _bool(v) -> bool:
    if isinstance(v, bool):
        return v
    return str(v).strip().lower() in ("1", "true", "yes", "on")


_PARSERS: Dict[str, Callable[[Any], Any]] = {
    "str": str, "int": lambda v: int(float(v)), "float": float, "bool": _bool,
    "bytes": lambda v: __import__("raydp_amd.utils", fromlist=["parse_memory_size"]).parse_memory_size(str(v)),
}


@dataclass
class ConfigKey:
    key: str
    type: str
    default: Any
    doc: str
    env: Optional[str] = None
    choices: Optional[List[str]] = None
    ignored: bool = False          # JVM-only knob: accepted, has no effect here
    prefix: bool = False           # the key is a prefix (``…resource.<name>``)
    ref: str = ""                  # where the reference declares / reads it
    aliases: List[str] = field(default_factory=list)

    def parse(self, raw):
        v = _PARSERS[self.type](raw)
        if self.choices is not None and v not in self.choices:
            raise ValueError(f"{self.key}={raw!r}: expected one of {self.choices}")
        return v


REGISTRY: Dict[str, ConfigKey] = {}


def register(key: str, type: str, default: Any, doc: str, **kw) -> ConfigKey:
    k = ConfigKey(key, type, default, doc, **kw)
    REGISTRY[key] = k
    for a in k.aliases:
        REGISTRY[a] = k
    return k


# ---------------------------------------------------------------- reference (RayDP) keys ----
_J = "core/raydp-main/src/main/java/org/apache/spark/raydp/SparkOnRayConfigs.java"
register("spark.executor.instances", "int", 1, "number of executor actors (init_spark num_executors)",
         ref="python/raydp/spark/ray_cluster.py:118")
register("spark.executor.cores", "int", 1, "task slots per executor (init_spark executor_cores)",
         ref="python/raydp/spark/ray_cluster.py:119")
register("spark.executor.memory", "bytes", "1g", "executor memory (init_spark executor_memory)",
         ref="python/raydp/spark/ray_cluster.py:120")
register("spark.ray.raydp_spark_executor.actor.resource.", "float", None,
         "runtime resources per executor actor; `cpu` sets the actor CPU (may oversubscribe)",
         prefix=True, ref=f"{_J}:8-9,36-37")
register("spark.ray.actor.resource.cpu", "float", None, "deprecated executor actor CPU",
         ref=f"{_J}:5-6,27-28")
register("spark.ray.raydp_spark_master.actor.resource.", "float", None,
         "resources of the master actor (CPU, memory, custom)", prefix=True,
         aliases=["spark.ray.raydp_spark_master.resource."], ref="python/raydp/spark/ray_cluster.py:80-98")
register("spark.ray.placement_group", "str", None, "internal: placement group id", ref="python/raydp/context.py:79")
register("spark.ray.bundle_indexes", "str", None, "internal: comma-separated bundle indexes",
         ref="python/raydp/context.py:80")
register("spark.ray.raydp_recoverable_fetch.task.resource.CPU", "float", 1.0,
         "CPU of each recoverable-conversion fetch task", ref="python/raydp/spark/dataset.py:195-200")
register("spark.ray.raydp_recoverable_fetch.task.resource.memory", "bytes", "0",
         "memory of each recoverable-conversion fetch task", ref="python/raydp/spark/dataset.py:195-200")
register("spark.shuffle.service.enabled", "bool", False,
         "start one external shuffle-block service per node (csrc/exec/shuffle_service.cc)",
         ref="core/raydp-main/src/main/scala/org/apache/spark/deploy/raydp/RayAppMaster.scala:155-163")
register("spark.local.dir", "str", None, "directory of spilled shuffle files",
         ref="core/raydp-main/src/main/scala/org/apache/spark/deploy/raydp/RayExternalShuffleService.scala:41-56")
register("spark.dynamicAllocation.enabled", "bool", False, "dynamic executor allocation",
         ref="core/raydp-main/src/main/scala/org/apache/spark/deploy/raydp/RayAppMaster.scala:275-288")
register("spark.dynamicAllocation.maxExecutors", "int", None, "upper bound under dynamic allocation",
         ref="python/raydp/spark/ray_cluster.py:167-175")
register("spark.dynamicAllocation.minExecutors", "int", 0, "lower bound under dynamic allocation")
register("spark.dynamicAllocation.initialExecutors", "int", None, "initial executors under dynamic allocation")
register("spark.driver.host", "str", None, "driver address (default: node IP)", ref="python/raydp/spark/ray_cluster.py:121-124")
register("spark.driver.bindAddress", "str", None, "driver bind address (default: node IP)")
register("spark.locality.wait", "str", "3s",
         "delay scheduling: how long a task waits for a slot on the node holding its input")
register("spark.task.maxFailures", "int", 4, "task attempts before a stage fails (executor loss)")
register("spark.sql.session.timeZone", "str", "UTC", "session time zone of datetime functions")
for _k, _r in [("spark.ray.raydp_app_master.extraJavaOptions", "python/raydp/spark/ray_cluster_master.py:116-119"),
               ("raydp.executor.extraClassPath", "python/raydp/spark/ray_cluster_master.py:93-95"),
               ("spark.javaagent", f"{_J}:55"), ("spark.ray.log4j.factory.class", f"{_J}:66"),
               ("spark.preferClassPath", f"{_J}:106"), ("spark.ray.preferClassPath", f"{_J}:114"),
               ("spark.log4j.config.file.name", "python/raydp/spark/ray_cluster_master.py:48"),
               ("spark.ray.log4j.config.file.name", f"{_J}:88"),
               ("spark.driver.extraClassPath", "python/raydp/spark/ray_cluster.py:160-189"),
               ("spark.driver.extraJavaOptions", "python/raydp/spark/ray_cluster.py:160-189"),
               ("spark.executor.extraJavaOptions", "")]:
    register(_k, "str", None, "JVM-only setting: accepted and ignored (no JVM here)", ignored=True, ref=_r)

# ---------------------------------------------------------------------- MI355X keys --------
register("spark.ray.mi355x.allreduce", "str", "auto",
         "gradient all-reduce of the fused trainer: auto (one-shot xGMI when every rank maps its "
         "peers, else RCCL), xgmi (required), rccl", env="RAYDP_ALLREDUCE", choices=["auto", "xgmi", "rccl"])
register("spark.ray.mi355x.allreduce.timeout_s", "float", 30.0,
         "bound on every xGMI flag wait before the kernel gives up and reports an error",
         env="RAYDP_ALLREDUCE_TIMEOUT_S")
register("spark.ray.mi355x.allreduce.oneshot_max_mb", "float", 16.0,
         "DDP / Horovod buckets up to this size take the xGMI kernels (one-shot or two-shot, see "
         "twoshot_min_mb); larger ones go to RCCL", env="RAYDP_ALLREDUCE_ONESHOT_MAX_MB")
register("spark.ray.mi355x.allreduce.twoshot_min_mb", "float", 1.0,
         "at world > 2, xGMI buckets from this size on take the two-shot kernel (all-pairs "
         "reduce-scatter + all-gather: 2S/N bytes per link, two flag rounds) instead of the one-shot "
         "kernel (S bytes per link, one flag round)", env="RAYDP_ALLREDUCE_TWOSHOT_MIN_MB")
register("spark.ray.mi355x.ddp.comm_stream", "str", "auto",
         "reduce DDP / Horovod gradient buckets on a dedicated comm stream, concurrent with the rest "
         "of backward (event fork/join: capturable): on, off, or auto = on when every rank of the "
         "group has a GPU of its own. Ranks sharing a GPU measured 5-8x slower with it (the early "
         "comm kernel spins for its peer on the CUs the peer's backward needs; "
         "profiles/r4_ddp_bucket_sweep.txt)", env="RAYDP_DDP_COMM_STREAM",
         choices=["auto", "on", "off", "true", "false", "1", "0"])
register("spark.ray.mi355x.fused", "str", "auto",
         "TorchEstimator engine: auto (fused HIP MLP when the model is an MLP), on (required), off",
         env="RAYDP_FUSED", choices=["auto", "on", "off"])
register("spark.ray.mi355x.hip_graphs", "bool", True, "replay torch training steps as HIP graphs",
         env="RAYDP_TORCH_GRAPHS")
register("spark.ray.mi355x.mlp_jit", "bool", True, "per-model specialised fused-MLP code objects",
         env="RAYDP_MLP_JIT")
register("spark.ray.mi355x.mlp_wgrad", "str", "opt",
         "fused MLP weight gradients: opt (computed by the optimizer kernel's workgroups from exported "
         "activations) or step (inside the single-workgroup step kernel)", env="RAYDP_MLP_WGRAD",
         choices=["opt", "step"])
register("spark.ray.mi355x.mlp_persistent", "bool", True,
         "one GPU: run a whole fused-MLP epoch as one persistent launch with the optimizer beside the "
         "backward pass (csrc/hip/mlp_persist.h)", env="RAYDP_MLP_PERSISTENT")
register("spark.ray.mi355x.fused_linear", "bool", True,
         "run Linear(+ReLU) towers of the DLRM-class models (TorchMlp) on the fused MFMA GEMM kernels "
         "(csrc/hip/linear_act.hip) instead of eager torch", env="RAYDP_FUSED_LINEAR")
register("spark.ray.mi355x.mlp_persistent.timeout_s", "float", 5.0,
         "bound on every workgroup hand-off wait of the persistent epoch kernel; on expiry the epoch "
         "is rolled back and rerun on the launch-per-step loop", env="RAYDP_MLP_PERSISTENT_TIMEOUT_S")
register("spark.ray.mi355x.driver_gc_freeze", "bool", True,
         "init_spark moves the driver's long-lived state (imported torch / pyarrow / engine modules, "
         "~180k objects) to the permanent GC generation, so a full collection no longer walks it "
         "(53-89 ms each, measured; raydp_amd/utils/gcmeter.py)", env="RAYDP_DRIVER_GC_FREEZE")
register("spark.ray.mi355x.ddp.bucket_mb", "float", 0.0,
         "DDP gradient bucket size in MiB; 0 = auto: when a bucket's all-reduce can run beside the rest "
         "of backward (comm stream on, or RCCL/gloo async on GPUs of their own) the first bucket is "
         "ddp.first_bucket_mb and the rest ddp.overlap_bucket_mb, so k buckets give k - 1 reductions "
         "that overlap backward; with the reduction stream-ordered (ranks sharing a GPU) nothing can "
         "overlap and 32 MiB buckets (few collectives) measured fastest (profiles/r4_ddp_bucket_sweep.txt)",
         env="RAYDP_DDP_BUCKET_MB")
register("spark.ray.mi355x.ddp.first_bucket_mb", "float", 1.0,
         "auto bucketing with overlap: size of the first bucket (the last layers' gradients, produced "
         "first by backward; small so its reduction starts early, as torch DDP's first bucket)",
         env="RAYDP_DDP_FIRST_BUCKET_MB")
register("spark.ray.mi355x.ddp.overlap_bucket_mb", "float", 4.0,
         "auto bucketing with overlap: size of every later bucket (large enough that one xGMI bucket's "
         "flag rendezvous is amortised over ~4 MiB of link traffic)", env="RAYDP_DDP_OVERLAP_BUCKET_MB")
register("spark.ray.mi355x.runtime.port", "int", -1,
         "TCP port of the head node's control endpoint (raydp_amd/runtime/gcs.py; 0 = any free port, "
         "-1 = Unix socket in the session directory only); a TCP client presents the session token",
         env="RAYDP_RUNTIME_PORT")
register("spark.ray.mi355x.runtime.host", "str", "127.0.0.1",
         "interface the control endpoint's TCP port binds to (loopback by default)", env="RAYDP_RUNTIME_HOST")
register("spark.ray.mi355x.object_store_bytes", "bytes", "0",
         "shared-memory object-store arena per node (0: automatic)", env="RAYDP_OBJECT_STORE_BYTES")
register("spark.ray.mi355x.trace", "str", None,
         "write a Chrome-trace JSON of runtime/ETL/training spans to this path", env="RAYDP_TRACE")
register("spark.ray.mi355x.roctx", "bool", False, "emit roctx ranges for every span (rocprofv3 --marker-trace)",
         env="RAYDP_ROCTX")
register("spark.ray.mi355x.opt_xcd_affine", "bool", True,
         "run the fused optimizer only on XCD 0's workgroups (the step kernel's L2)", env="RAYDP_OPT_XCD_AFFINE")
register("spark.ray.mi355x.fused_etl", "bool", True,
         "run chains of filter/withColumn/select/drop as one native expression-VM program per partition "
         "(csrc/exec/expr/expr_vm.cc)", env="RAYDP_FUSED_ETL")
register("spark.ray.mi355x.local_exec_bytes", "bytes", "4m",
         "stages whose inputs are driver-resident tables (cached / local data) below this size run in "
         "the driver process instead of on executors (0: never)", env="RAYDP_LOCAL_EXEC_BYTES")
register("spark.ray.mi355x.xg_opt_stride", "int", 1,
         "workgroup stride of the fused reduce+optimizer kernel (1: every XCD pulls peer lines)",
         env="RAYDP_XG_OPT_STRIDE")
register("spark.ray.mi355x.step_times", "bool", True,
         "record the device time of every fused-MLP step (one store per step) and report a step-time "
         "histogram with each epoch", env="RAYDP_STEP_TIMES")
register("spark.ray.mi355x.udf_verify", "str", "sampled",
         "inlined Python UDFs: sampled (spread rows + every argument's new extreme rows per partition) "
         "or full (every row checked against the Python function)", env="RAYDP_UDF_VERIFY",
         choices=["sampled", "full"])
register("spark.ray.mi355x.native_executor", "bool", True,
         "executors run persisted stages whose operators all lower to the expression VM on the native "
         "task loop (csrc/exec/executor.cc: CSV split or Arrow stream -> VM -> IPC straight into the "
         "object store); other stages and fallback partitions take the Python path",
         env="RAYDP_NATIVE_EXECUTOR")
register("spark.ray.mi355x.overlap_conversion", "bool", True,
         "fit_on_spark: the training engine is built (device buffers, kernels, parameter upload) while "
         "the conversion stage runs on the executors; the dataset blocks are awaited at first use",
         env="RAYDP_OVERLAP_CONVERSION")

register("spark.ray.mi355x.fused_optimizer", "bool", True,
         "Horovod's DistributedOptimizer, and a torch Adam / AdamW / SGD stepped in a GPU train worker's "
         "loop (raydp_amd/train/gpu_policy.py fused_optimizers), run the step on the multi-tensor HIP "
         "kernels (csrc/hip/fused_optim.hip: one launch per 24 tensors) when every parameter is a dense "
         "fp32 GPU tensor; torch's own step otherwise (closures, step hooks, graph capture, amsgrad / "
         "capturable / fused groups)", env="RAYDP_FUSED_OPTIMIZER")
register("spark.ray.mi355x.native_batchnorm", "bool", True,
         "GPU train workers run BatchNorm layers on PyTorch's native kernels instead of MIOpen's (MIOpen's "
         "batch-norm path is launch-bound at tabular batch sizes: scripts/dev/eager_step_bench.py, "
         "profiles/r5_eager_variants.jsonl); only the BatchNorm call is affected, convolutions keep MIOpen",
         env="RAYDP_NATIVE_BATCHNORM")

register("spark.ray.mi355x.graph_user_model", "bool", True,
         "train.torch.prepare_model on a one-worker GPU job replays the model's training forward + "
         "backward as HIP graphs per repeated batch shape (raydp_amd/train/gpu_policy.py graph_model); "
         "eager for eval, other shapes and models that cannot be captured", env="RAYDP_GRAPH_USER_MODEL")

register("spark.ray.mi355x.graph_hvd_model", "bool", False,
         "hvd.DistributedOptimizer(named_parameters=model.named_parameters()) also applies the "
         "graph_user_model policy to that module (raydp_amd/hvd/__init__.py _graph_user_module): the "
         "Horovod NYC step goes from ~0.9 to ~0.46 ms once captured, but the first capture in a process "
         "costs ~0.4 s, which a short fit never earns back; off by default", env="RAYDP_GRAPH_HVD_MODEL")

register("spark.ray.mi355x.stream_ingest", "bool", True,
         "fit_on_spark with one in-process worker: the fused engine DMAs each training block into HBM as "
         "its conversion task lands, while the rest of the stage runs (raydp_amd/torch/engine.py "
         "stream_ingest)", env="RAYDP_STREAM_INGEST")

register("spark.ray.mi355x.train_inprocess", "bool", True,
         "a one-worker fit runs its loop in the caller's process (no worker hop); off: through a "
         "spawned worker actor, as Ray Train always does (the bench's N = 1 worker-hop measurement)",
         env="RAYDP_TRAIN_INPROCESS")


def _active_conf() -> Optional[Mapping]:
    try:
        from raydp_amd.spark import session as S
        s = S._active_session
        if s is not None and not s._stopped:
            return s.conf
    except Exception:  # noqa: BLE001
        return None
    return None


def _lookup(m, key):
    if m is None:
        return None
    try:
        return m.get(key, None)
    except TypeError:
        return m.get(key)


def lookup(key: str) -> ConfigKey:
    if key in REGISTRY:
        return REGISTRY[key]
    for name, k in REGISTRY.items():
        if k.prefix and key.startswith(name):
            return k
    raise KeyError(f"unknown configuration key {key!r}")


def get(key: str, conf: Optional[Mapping] = None, default: Any = None):
    """Typed value of ``key`` (see module doc for precedence)."""
    k = lookup(key)
    for src in (conf, _active_conf()):
        raw = _lookup(src, key)
        if raw is not None:
            return k.parse(raw)
    if k.env and os.environ.get(k.env) not in (None, ""):
        return k.parse(os.environ[k.env])
    if default is not None:
        return default
    return k.parse(k.default) if k.default is not None else None


def with_prefix(prefix: str, conf: Mapping) -> Dict[str, Any]:
    """``{suffix: typed value}`` of every ``prefix<suffix>`` entry of ``conf``."""
    k = lookup(prefix)
    items = conf.items() if hasattr(conf, "items") else conf.getAll()
    return {kk[len(prefix):]: k.parse(v) for kk, v in items if kk.startswith(prefix)}


def validate(conf: Mapping) -> List[str]:
    """Check every registered key of ``conf``; returns the ignored (JVM-only) keys set."""
    items = conf.items() if hasattr(conf, "items") else conf
    ignored = []
    for key, raw in items:
        try:
            k = lookup(key)
        except KeyError:
            continue  # free-form Spark keys stay allowed
        if k.ignored:
            log.debug("configuration %s has no effect (JVM-only)", key)
            ignored.append(key)
            continue
        k.parse(raw)
    return ignored


def env_for_workers(conf: Optional[Mapping] = None) -> Dict[str, str]:
    """Environment that carries every set MI355X key into worker processes."""
    out = {}
    for k in {id(v): v for v in REGISTRY.values()}.values():
        if not k.env:
            continue
        v = _lookup(conf, k.key) if conf is not None else None
        if v is None:
            v = _lookup(_active_conf(), k.key)
        if v is not None:
            out[k.env] = str(v)
    return out


def describe(keys: Iterable[str] = None) -> str:
    """Markdown table of the registry (docs)."""
    rows = ["| key | type | default | env | meaning |", "|---|---|---|---|---|"]
    seen = set()
    for k in REGISTRY.values():
        if id(k) in seen or (keys is not None and k.key not in keys):
            continue
        seen.add(id(k))
        rows.append(f"| `{k.key}` | {k.type} | {k.default} | {k.env or ''} | "
                    f"{'(ignored) ' if k.ignored else ''}{k.doc} |")
    return "\n".join(rows)
