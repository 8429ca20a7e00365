"""Build the in-tree native libraries.

* ``libexec_kernels.so``  — CPU shuffle/hash kernels (g++).
* ``libraydp_runtime.so`` — shared-memory object store + actor supervisor + framed IPC (g++).
* ``libhipkernels.so``    — CDNA4 HIP kernels for gfx950 (hipcc ``--offload-arch=gfx950``).
* ``raydp_supervisor`` / ``raydp_appmaster`` / ``raydp_shuffle_service`` — native services (g++).

``build_sanitized("asan"|"tsan", dir)`` builds the host-side services and the runtime stress
test under AddressSanitizer+UBSan or ThreadSanitizer (``scripts/sanitize_runtime.sh``).

Usage: ``python -m raydp_amd.native.build [name ...]``.
"""
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
CSRC = os.path.join(ROOT, "csrc")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("RAYDP_GPU_ARCH", "gfx950")


def _hip_sources():
    d = os.path.join(CSRC, "hip")
    c = os.path.join(CSRC, "comm")
    srcs = sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".hip"))
    if os.path.isdir(c):
        srcs += sorted(os.path.join(c, f) for f in os.listdir(c) if f.endswith((".cc", ".hip")))
    return srcs


def _runtime_sources():
    d = os.path.join(CSRC, "runtime")
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".cc") and f not in _EXE_SOURCES)


_EXE_SOURCES = {"supervisor.cc"}


LIBS = {
    "exec_kernels": dict(kind="cpu", sources=lambda: [os.path.join(CSRC, "exec", "exec_kernels.cc"),
                                                       os.path.join(CSRC, "exec", "expr", "expr_vm.cc")]),
    "raydp_runtime": dict(kind="cpu", sources=_runtime_sources, libs=["-lpthread", "-lrt", "-ldl"]),
    # native executor core: task loop, CSV/stream sources, VM segments, IPC sink into the
    # object store, partition cache (Arrow C++ from the pyarrow wheel; libraydp_runtime)
    "raydp_executor": dict(kind="cpu", std="c++20", arrow=True,
                           sources=lambda: [os.path.join(CSRC, "exec", "executor.cc"),
                                            os.path.join(CSRC, "exec", "csv_infer.cc"),
                                            os.path.join(CSRC, "exec", "expr", "expr_vm.cc")],
                           libs=["-L", HERE, "-lraydp_runtime", "-Wl,-rpath,$ORIGIN", "-lpthread"]),
    "hipkernels": dict(kind="hip", sources=_hip_sources),
    # executables: the per-node actor supervisor, the application master (native control
    # plane) and the per-node external shuffle-block service
    "raydp_supervisor": dict(kind="exe", sources=lambda: [os.path.join(CSRC, "runtime", "supervisor.cc")]),
    "raydp_appmaster": dict(kind="exe", sources=lambda: [os.path.join(CSRC, "control", "app_master.cc")]),
    "raydp_shuffle_service": dict(kind="exe", sources=lambda: [os.path.join(CSRC, "exec", "shuffle_service.cc")]),
}


def _arrow_flags():
    """Compile/link flags for Arrow C++ as shipped in the pyarrow wheel: the executor library
    links the SAME libarrow the Python process already has loaded (one memory pool, one
    type registry)."""
    import pyarrow as pa
    libdir = pa.get_library_dirs()[0]
    so = sorted(f for f in os.listdir(libdir) if f.startswith("libarrow.so."))
    if not so:
        raise RuntimeError(f"no libarrow.so.* under {libdir}")
    return ["-I", pa.get_include(), "-L", libdir, f"-l:{so[0]}", f"-Wl,-rpath,{libdir}"]


def out_path(name: str) -> str:
    return os.path.join(HERE, name if LIBS[name]["kind"] == "exe" else f"lib{name}.so")


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _newer(out, srcs):
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    deps = list(srcs)
    for d in ("common", "hip", "runtime", "exec", "exec/expr", "comm", "control"):
        p = os.path.join(CSRC, d)
        if os.path.isdir(p):
            deps += [os.path.join(p, f) for f in os.listdir(p) if f.endswith((".h", ".hpp", ".cuh"))]
    return all(os.path.getmtime(s) <= t for s in deps)


def build_one(name: str, force: bool = False) -> str:
    spec = LIBS[name]
    srcs = spec["sources"]()
    out = out_path(name)
    if not force and _newer(out, srcs):
        return out
    tmp = out + f".tmp{os.getpid()}"
    inc = ["-I", os.path.join(CSRC, "common"), "-I", CSRC]
    if spec["kind"] == "exe":
        cxx = shutil.which("g++") or "c++"
        _run([cxx, "-O2", "-std=c++17", "-Wall"] + inc + srcs + ["-o", tmp])
    elif spec["kind"] == "cpu":
        cxx = shutil.which("g++") or "c++"
        extra = _arrow_flags() if spec.get("arrow") else []
        cmd = [cxx, "-O3", f"-std={spec.get('std', 'c++17')}", "-shared", "-fPIC", "-Wall",
               "-Wno-unused-function"] + inc + srcs + ["-o", tmp] + spec.get("libs", []) + extra
        _run(cmd)
    else:
        hipcc = os.path.join(ROCM, "bin", "hipcc")
        # one object per source, kept between builds (a source is recompiled when it or any
        # header is newer than its object) and compiled in parallel
        od = os.path.join(os.path.dirname(CSRC), "build", "hipobj")
        os.makedirs(od, exist_ok=True)
        objs = [os.path.join(od, os.path.basename(s) + ".o") for s in srcs]
        todo = [(s, o) for s, o in zip(srcs, objs) if force or not _newer(o, [s])]
        from concurrent.futures import ThreadPoolExecutor
        jobs = max(1, min(len(todo), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
        def compile_one(so):
            src, obj = so
            _run([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
                  "-c", src, "-o", obj + ".tmp"] + inc)
            os.replace(obj + ".tmp", obj)

        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(compile_one, todo))
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC"] + objs + ["-o", tmp, "-ldl"])
    os.replace(tmp, out)
    return out


SANITIZERS = {"asan": ["-fsanitize=address,undefined,float-cast-overflow", "-fno-omit-frame-pointer",
                        "-fno-sanitize-recover=undefined,float-cast-overflow"],
              "tsan": ["-fsanitize=thread"]}


def build_sanitized(kind: str, out_dir: str, names=("raydp_supervisor", "raydp_appmaster", "raydp_shuffle_service"),
                    stress: bool = True) -> dict:
    """Host C++ (services + the runtime stress test) under a sanitizer, into ``out_dir``
    (SURVEY.md §5.2). Returns ``{name: path}``."""
    flags = SANITIZERS[kind]
    os.makedirs(out_dir, exist_ok=True)
    cxx = shutil.which("g++") or "c++"
    inc = ["-I", os.path.join(CSRC, "common"), "-I", CSRC]
    out = {}
    for n in names:
        p = os.path.join(out_dir, n)
        _run([cxx, "-O1", "-g", "-std=c++17", "-Wall"] + flags + inc + LIBS[n]["sources"]() + ["-o", p])
        out[n] = p
    if stress:
        p = os.path.join(out_dir, "runtime_stress")
        _run([cxx, "-O1", "-g", "-std=c++17"] + flags + inc +
             [os.path.join(CSRC, "tests", "runtime_stress.cc"), os.path.join(CSRC, "runtime", "objstore.cc"),
              "-o", p, "-lpthread", "-lrt"])
        out["runtime_stress"] = p
        # random well-typed programs through the fused expression VM (adversarial values)
        p = os.path.join(out_dir, "expr_vm_fuzz")
        _run([cxx, "-O1", "-g", "-std=c++17"] + flags + inc +
             [os.path.join(CSRC, "tests", "expr_vm_fuzz.cc"), os.path.join(CSRC, "exec", "expr", "expr_vm.cc"),
              "-o", p])
        out["expr_vm_fuzz"] = p
        # the native executor core: task loop + partition cache + CSV reader, many threads
        p = os.path.join(out_dir, "executor_stress")
        _run([cxx, "-O1", "-g", "-std=c++20"] + flags + inc +
             [os.path.join(CSRC, "tests", "executor_stress.cc"), os.path.join(CSRC, "exec", "executor.cc"),
              os.path.join(CSRC, "exec", "csv_infer.cc"), os.path.join(CSRC, "exec", "expr", "expr_vm.cc"),
              os.path.join(CSRC, "runtime", "objstore.cc"), "-o", p, "-lpthread", "-lrt"] + _arrow_flags())
        out["executor_stress"] = p
    return out


def build_all(names=None, force=False):
    for n in names or LIBS:
        if LIBS[n]["kind"] == "hip" and not os.path.exists(os.path.join(ROCM, "bin", "hipcc")):
            raise RuntimeError("hipcc not found; cannot build the gfx950 kernels")
        if not LIBS[n]["sources"]():
            continue
        p = build_one(n, force=force)
        print(f"built {p}")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("-")]
    if "--sanitize" in sys.argv:  # python -m raydp_amd.native.build --sanitize asan <dir>
        print(build_sanitized(args[0], args[1]))
    else:
        build_all(args or None, force="--force" in sys.argv)
