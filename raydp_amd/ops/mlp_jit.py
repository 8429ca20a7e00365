"""Per-model specialised fused-MLP step kernels.

``FusedMLPTrainer`` describes its network with an ``MlpDesc`` (layer dims, paddings, LDS and
buffer offsets, loss). The ahead-of-time kernel reads that descriptor from device memory at
run time; this module instead *generates* a translation unit in which every one of those
numbers is a compile-time constant (empty structs with ``static constexpr`` members, consumed
by the same device code in ``csrc/hip/mlp_core.h``), compiles it for gfx950 with
``hipcc --genco`` and loads the code object with ``hipModuleLoad``. With the layer loop
unrolled and all offsets known, the compiler schedules each layer's loads, MFMAs and
epilogue as straight-line code (no descriptor loads, no dead branches, exact trip counts).

Code objects are cached by content hash under ``raydp_amd/native/jit/`` (in-tree, so a cache
warmed by ``__graft_entry__.build()`` travels with the repository); a cold cache costs one
hipcc run (~10-20 s) per distinct model/loss/batch-size.
"""
import ctypes
import hashlib
import os
import subprocess
import threading
from typing import Optional

from raydp_amd.ops import _hip

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
CSRC_HIP = os.path.join(ROOT, "csrc", "hip")
CACHE = os.environ.get("RAYDP_JIT_CACHE", os.path.join(ROOT, "raydp_amd", "native", "jit"))
ARCH = os.environ.get("RAYDP_GPU_ARCH", "gfx950")
_lock = threading.Lock()
_loaded = {}

_LAYER_INT = ("in_", "out", "in_k", "out_k", "in_n", "out_n", "w_img", "wt_img", "w_off", "b_off", "act", "bn",
              "g_off", "be_off", "rs_off", "xt_off", "stat_off", "r_off", "pr_off", "xg_off", "gg_off", "mw_off",
              "sv_lds")
_DESC_INT = ("L", "r_lds_off", "gt_lds_off", "stats_lds_off", "lds_bytes", "max_k", "max_n", "loss", "out_dim",
             "feat_k", "pr_lds_off", "pr_total", "act_off", "wgrad_mode", "front_n", "front_q", "acc_mode",
             "loss_lds_off", "w0s_lds_off", "x0c_lds_off")


def _f(x: float) -> str:
    return repr(float(x)) + "f" if "e" in repr(float(x)) or "." in repr(float(x)) else f"{float(x)}f"


def generate_source(desc: "_hip.MlpDesc", mt: int, opt: Optional["_hip.OptDesc"] = None,
                    xg: bool = True) -> str:
    """``opt``: the optimizer's hyperparameters become constants too (the persistent kernel's
    in-epilogue bias / BatchNorm updates, csrc/hip/mlp_core.h PsVec). ``xg`` False (a one-GPU
    trainer): the in-launch gradient exchange is compiled out (csrc/comm/xgmi.h RX_XG_KERNELS)."""
    L = desc.L
    out = [] if xg else ["#define RX_XG_KERNELS 0"]
    if os.environ.get("RAYDP_MLP_LAYER_STAMPS") == "1":
        # diagnostic build: the persistent epoch's middle step writes intra-layer s_memtime stamps
        out.append("#define RX_LAYER_STAMPS 1")
    for dfn in os.environ.get("RAYDP_MLP_DEFINES", "").split():
        # dev A/B builds: NAME or NAME=VALUE macros for kernel variants measured side by side
        name, _, val = dfn.partition("=")
        if name.isidentifier():
            out.append(f"#define {name} {val or 1}")
    out += ['#include "mlp_persist.h"', "", "namespace {", "", "struct JD {"]
    for k in _DESC_INT:
        out.append(f"  static constexpr int {k} = {int(getattr(desc, k))};")
    out.append(f"  static constexpr float beta = {_f(desc.beta)};")
    out.append(f"  static constexpr float acc_thr = {_f(desc.acc_thr)};")
    out.append("};")
    for li in range(L):
        ly = desc.layer[li]
        out.append(f"struct JL{li} {{")
        for k in _LAYER_INT:
            out.append(f"  static constexpr int {k.rstrip('_')} = {int(getattr(ly, k))};")
        out.append(f"  static constexpr float eps = {_f(ly.eps)};")
        out.append(f"  static constexpr float momentum = {_f(ly.momentum)};")
        out.append("};")
    if opt is not None:
        out.append("struct JO {")
        for k in ("algo", "nesterov", "maximize"):
            out.append(f"  static constexpr int {k} = {int(getattr(opt, k))};")
        for k in ("b1", "b2", "eps", "wd", "momentum", "dampening"):
            out.append(f"  static constexpr float {k} = {_f(getattr(opt, k))};")
        out.append("};")
    fwd = "; ".join(f"f(JL{li}{{}}, JL{min(li + 1, L - 1)}{{}}, {li}, {'true' if li == L - 1 else 'false'})"
                    for li in range(L))
    bwd = "; ".join(f"f(JL{li}{{}}, JL{max(li - 1, 0)}{{}}, {li})" for li in range(L - 1, -1, -1))
    each = "; ".join(f"f(JL{li}{{}}, {li})" for li in range(L))
    out += [
        "struct JitCfg {",
        *(["  using Opt = JO;"] if opt is not None else []),
        "  __device__ static JD desc(const MlpDesc*) { return {}; }",
        f"  template <class F> __device__ static void fwd_layers(const JD&, F&& f) {{ {fwd}; }}",
        f"  template <class F> __device__ static void bwd_layers(const JD&, F&& f) {{ {bwd}; }}",
        f"  template <class F> __device__ static void each_layer(const JD&, F&& f) {{ {each}; }}",
        "  __device__ static JL0 first(const JD&) { return {}; }",
        "};",
        "}  // namespace",
        "",
        f"#define RX_MT {mt}",
        'extern "C" __global__ __launch_bounds__(RX_THREADS) void rx_jit_step(',
        "    const MlpDesc* __restrict__ dp, const u16* __restrict__ img, float* __restrict__ rstats,",
        "    const float* __restrict__ P, float* __restrict__ Gr, const u16* __restrict__ feats,",
        "    const float* __restrict__ labels, const int* __restrict__ perm, int row0, int nvalid,",
        "    float* __restrict__ scratch, double* __restrict__ metrics, unsigned long long* __restrict__ stamps) {",
        "  extern __shared__ __attribute__((aligned(16))) char smem[];",
        "  __shared__ int rowidx[Tile<RX_MT>::BP];",
        "  mlp_train_step_body<JitCfg, RX_MT>(dp, img, rstats, P, Gr, feats, labels, perm, row0, nvalid, scratch,",
        "                                     metrics, stamps, smem, rowidx);",
        "}",
        'extern "C" __global__ __launch_bounds__(RX_THREADS) void rx_jit_step_mw(',
        "    const MlpDesc* __restrict__ dp, const u16* __restrict__ img, float* __restrict__ rstats,",
        "    const float* __restrict__ P, float* __restrict__ Gr, const u16* __restrict__ feats,",
        "    const float* __restrict__ labels, const int* __restrict__ perm, int row0, float* __restrict__ scratch,",
        "    long long scratch_stride, double* __restrict__ metrics, MwCtx mw) {",
        "  extern __shared__ __attribute__((aligned(16))) char smem[];",
        "  __shared__ int rowidx[Tile<RX_MT>::BP];",
        "  mlp_train_step_mw_body<JitCfg, RX_MT>(dp, img, rstats, P, Gr, feats, labels, perm, row0, scratch,",
        "                                        scratch_stride, metrics, mw, smem, rowidx);",
        "}",
        'extern "C" __global__ __launch_bounds__(RX_THREADS) void rx_jit_eval(',
        "    const MlpDesc* __restrict__ dp, const u16* __restrict__ img, const float* __restrict__ rstats,",
        "    const float* __restrict__ P, const u16* __restrict__ feats, const float* __restrict__ labels,",
        "    int n_rows, int batch, double* __restrict__ metrics) {",
        "  extern __shared__ __attribute__((aligned(16))) char smem[];",
        "  __shared__ int rowidx[Tile<RX_MT>::BP];",
        "  mlp_eval_body<JitCfg, RX_MT>(dp, img, rstats, P, feats, labels, n_rows, batch, metrics, smem, rowidx);",
        "}",
        'extern "C" __global__ __launch_bounds__(RX_THREADS) void rx_jit_persist(',
        "    const MlpDesc* __restrict__ dp, const OptDesc* __restrict__ od, const u16* __restrict__ img,",
        "    float* __restrict__ rstats, float* __restrict__ P, float* __restrict__ Gr,",
        "    const u16* __restrict__ feats, const float* __restrict__ labels, const int* __restrict__ perm,",
        "    int n_rows, int batch, int nsteps, float* __restrict__ scratch, double* __restrict__ metrics,",
        "    float* __restrict__ m, float* __restrict__ v, const float* __restrict__ sched, int opt_first,",
        "    unsigned* __restrict__ sync, unsigned long long ticks, unsigned long long* __restrict__ stamps,",
        "    XgStep xs) {",
        "  extern __shared__ __attribute__((aligned(16))) char smem[];",
        "  __shared__ int rowidx[Tile<RX_MT>::BP];",
        "  __shared__ __attribute__((aligned(16))) int flag_lds[16];",
        "  mlp_persist_body<JitCfg, RX_MT>(dp, od, img, rstats, P, Gr, feats, labels, perm, n_rows, batch, nsteps,",
        "                                  scratch, metrics, m, v, sched, opt_first, sync, ticks, smem, rowidx,",
        "                                  flag_lds, stamps, xs);",
        "}",
    ]
    return "\n".join(out) + "\n"


def _hipcc() -> str:
    return os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


_headers_digest = None


def _key(src: str) -> str:
    global _headers_digest
    if _headers_digest is None:      # the kernel headers a process compiles against: read once
        h = hashlib.sha256()
        for f in ("mlp_core.h", "mlp_opt.h", "mlp_mwopt.h", "mlp_persist.h", "rx_common.h", "rx_grid.h",
                  os.path.join("..", "comm", "xgmi.h")):
            with open(os.path.join(CSRC_HIP, f), "rb") as fh:
                h.update(fh.read())
        h.update(ARCH.encode())
        _headers_digest = h.digest()
    h = hashlib.sha256(src.encode())
    h.update(_headers_digest)
    return h.hexdigest()[:24]


def compile_source(src: str) -> str:
    """Compile (or find in the cache) the code object for ``src``; returns its path."""
    key = _key(src)
    path = os.path.join(CACHE, f"mlp_{key}.hsaco")
    if os.path.exists(path):
        try:
            os.utime(path)      # (used: a cache pruned by age keeps it)
        except OSError:
            pass
        return path
    os.makedirs(CACHE, exist_ok=True)
    cpp = os.path.join(CACHE, f"mlp_{key}.hip")
    with open(cpp + f".{threading.get_ident()}", "w") as f:
        f.write(src)
    os.replace(cpp + f".{threading.get_ident()}", cpp)
    tmp = path + f".tmp{os.getpid()}.{threading.get_ident()}"   # (precompile_many: same source twice)
    cmd = [_hipcc(), "--genco", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-munsafe-fp-atomics",
           "-I", CSRC_HIP, cpp, "-o", tmp]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"specialised kernel build failed:\n{' '.join(cmd)}\n{r.stdout[-4000:]}")
    os.replace(tmp, path)
    return path


_paths = {}     # (descriptor bytes, MT) -> code-object path: a refit of the same model shape
               # neither regenerates nor re-hashes the specialised source


_OPT_CONSTS = ("algo", "nesterov", "maximize", "b1", "b2", "eps", "wd", "momentum", "dampening")


def compile_for(trainer) -> str:
    opt = getattr(trainer, "opt", None)
    # (the optimizer descriptor also holds this fit's device pointers to the bf16 images: the key
    # takes only the fields the generated source reads, so a refit finds its code object here
    # instead of regenerating and hashing the source)
    xg = int(getattr(trainer, "world", 1)) > 1
    k = (bytes(trainer.desc), int(trainer.mt),
         tuple(getattr(opt, f) for f in _OPT_CONSTS) if opt is not None else (), xg)
    path = _paths.get(k)
    if path is None or not os.path.exists(path):
        path = compile_source(generate_source(trainer.desc, trainer.mt, opt, xg=xg))
        _paths[k] = path
    return path


def load_specialized(trainer) -> Optional[str]:
    """Compile/load the specialised kernels for ``trainer`` and plug them into its buffers."""
    path = compile_for(trainer)
    with _lock:
        fns = _loaded.get(path)
        if fns is None:
            step, ev, ps, mw = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
            _hip.check(_hip.lib().rx_jit_load(path.encode(), ctypes.byref(step), ctypes.byref(ev), ctypes.byref(ps),
                                              ctypes.byref(mw), int(trainer.desc.lds_bytes)), "rx_jit_load")
            fns = (step.value, ev.value, ps.value, mw.value)
            if not _loaded:
                import atexit
                atexit.register(_unload_all)
            _loaded[path] = fns
    trainer.bufs.jit_step, trainer.bufs.jit_eval, trainer.bufs.jit_persist, trainer.bufs.jit_step_mw = fns
    return path


def _unload_all():
    """Interpreter exit: wait for the device, then unload the specialised modules (before the HIP
    runtime's own teardown, which a profiling tool may already have finalised)."""
    try:
        import torch
        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
        with _lock:
            _hip.lib().rx_jit_unload_all()
            _loaded.clear()
    except Exception:  # noqa: BLE001 - best effort at exit
        pass


def precompile(model, optimizer, loss, batch_size: int, acc_thr=None) -> str:
    """Warm the code-object cache for one model/optimizer/loss/batch on a host without a GPU."""
    from raydp_amd.models.mlp_spec import extract_mlp_spec
    from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
    tr = FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(optimizer), loss_code(loss), batch_size,
                         None, layout_only=True, acc_thr=acc_thr)
    return compile_for(tr)


def precompile_many(jobs, workers: Optional[int] = None):
    """``precompile`` over ``[(model, optimizer, loss, batch_size, acc_thr[, world]), ...]``: the
    layouts are derived one after the other (spec extraction runs the model), the hipcc builds in
    parallel. ``world`` > 1: the data-parallel layout (layer 0 on optimizer workgroups). Returns
    the code-object paths."""
    from concurrent.futures import ThreadPoolExecutor
    from raydp_amd.models.mlp_spec import extract_mlp_spec
    from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
    trs = [FusedMLPTrainer(extract_mlp_spec(j[0]), optimizer_config(j[1]), loss_code(j[2]), j[3], None,
                           layout_only=True, acc_thr=j[4], world=j[5] if len(j) > 5 else 1) for j in jobs]
    n = workers or max(1, min(8, os.cpu_count() or 1))
    with ThreadPoolExecutor(n) as ex:
        return list(ex.map(compile_for, trs))
