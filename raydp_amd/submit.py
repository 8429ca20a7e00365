"""``raydp-submit``: run a PySpark application on the runtime (reference: ``bin/raydp-submit``
plus the forked ``SparkSubmit.scala`` / ``DependencyUtils.scala`` and the ``--master ray``
branch of ``RayCoarseGrainedSchedulerBackend.scala:81-117``).

    raydp-submit [--ray-conf FILE] [spark-submit options] app.py [app args]

Supported spark-submit options: ``--conf k=v`` (repeatable), ``--properties-file``,
``--name``, ``--num-executors``, ``--executor-cores``, ``--executor-memory``,
``--driver-memory``, ``--py-files`` (zip/egg/py, comma separated: added to the import path of the
driver and, through ``PYTHONPATH``, of every executor process), ``--files``, ``--master``
(``ray``; anything else is rejected), ``--deploy-mode client`` and ``--verbose``. JVM-only
options (``--jars``, ``--packages``, ``--driver-class-path``, ``--class``) are accepted and
ignored with a warning where they have no meaning without a JVM; a ``--class`` application
(a jar) cannot run and is an error.

``--ray-conf`` is the JSON file the reference writes (``{"ray": {"address": ..., ...}}``): an
``address`` (``raydp://<session dir>``, ``auto``, or ``host:port?token=...``) runs the application
against that running node (``raydp_amd/runtime/gcs.py``); without one, ``num-cpus`` /
``object-store-memory`` / ``namespace`` size a fresh local runtime.

The application runs in this process (as ``__main__``); its ``SparkSession.builder
.getOrCreate()`` sees ``spark.master=ray`` and starts executor processes with the submitted
confs. The runtime is shut down when the application returns.
"""
import json
import os
import runpy
import shutil
import sys
import tempfile
from typing import Dict, List, Tuple

_WITH_VALUE = {"--conf", "--properties-file", "--name", "--num-executors", "--executor-cores",
               "--executor-memory", "--driver-memory", "--driver-cores", "--py-files", "--files", "--jars",
               "--packages", "--repositories", "--exclude-packages", "--driver-class-path",
               "--driver-java-options", "--driver-library-path", "--class", "--master", "--deploy-mode",
               "--ray-conf", "--archives", "--total-executor-cores", "--queue", "--principal", "--keytab"}
_FLAGS = {"--verbose", "-v", "--supervise"}
_SHORTHAND = {"--name": "spark.app.name", "--num-executors": "spark.executor.instances",
              "--executor-cores": "spark.executor.cores", "--executor-memory": "spark.executor.memory",
              "--driver-memory": "spark.driver.memory", "--driver-cores": "spark.driver.cores",
              "--files": "spark.files", "--py-files": "spark.submit.pyFiles",
              "--archives": "spark.archives"}
_JVM_ONLY = {"--jars", "--packages", "--repositories", "--exclude-packages", "--driver-class-path",
             "--driver-java-options", "--driver-library-path"}


class SubmitError(ValueError):
    pass


def parse_args(argv: List[str]) -> Tuple[Dict[str, str], dict, str, List[str]]:
    """-> (spark confs, options, primary resource, app args)."""
    confs: Dict[str, str] = {}
    opts = {"verbose": False, "ray_conf": None, "warnings": []}
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in _FLAGS:
            opts["verbose"] = True
            i += 1
            continue
        key, val = a, None
        if "=" in a and a.split("=", 1)[0] in _WITH_VALUE:
            key, val = a.split("=", 1)
        if key in _WITH_VALUE:
            if val is None:
                if i + 1 >= len(argv):
                    raise SubmitError(f"missing value for {key}")
                val = argv[i + 1]
                i += 2
            else:
                i += 1
            if key == "--conf":
                if "=" not in val:
                    raise SubmitError(f"--conf expects key=value, got {val!r}")
                k, v = val.split("=", 1)
                confs[k] = v
            elif key == "--properties-file":
                confs.update({k: v for k, v in _read_properties(val).items() if k not in confs})
            elif key == "--ray-conf":
                opts["ray_conf"] = val
            elif key == "--master":
                if not (val == "ray" or val.startswith("ray://")):
                    raise SubmitError(f"raydp-submit runs on the ray master only (got --master {val})")
            elif key == "--deploy-mode":
                if val != "client":
                    raise SubmitError("only --deploy-mode client is supported")
            elif key == "--class":
                raise SubmitError("--class (JVM applications) is not supported: submit a Python application")
            elif key in _JVM_ONLY:
                opts["warnings"].append(f"{key} {val} ignored (no JVM)")
            elif key in _SHORTHAND:
                confs[_SHORTHAND[key]] = val
            continue
        if a.startswith("-"):
            raise SubmitError(f"unknown option {a}")
        return confs, opts, a, argv[i + 1:]
    raise SubmitError("no application file given")


def _read_properties(path: str) -> Dict[str, str]:
    out = {}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            if "=" in line:
                k, v = line.split("=", 1)
            else:
                parts = line.split(None, 1)
                k, v = parts[0], parts[1] if len(parts) > 1 else ""
            out[k.strip()] = v.strip()
    return out


def _runtime_kwargs(ray_conf_path) -> dict:
    if not ray_conf_path:
        return {}
    with open(ray_conf_path) as f:
        conf = json.load(f).get("ray", {})
    kw = {}
    if conf.get("address"):
        # run against the caller's running node (doc/spark_on_ray.md:116-144 of the reference)
        kw["address"] = str(conf["address"])
    if "num-cpus" in conf:
        kw["num_cpus"] = int(conf["num-cpus"])
    if "object-store-memory" in conf:
        kw["object_store_memory"] = int(conf["object-store-memory"])
    if "namespace" in conf:
        kw["namespace"] = conf["namespace"]
    return kw


def _stage_py_files(spec: str, workdir: str) -> List[str]:
    paths = []
    for item in [p for p in spec.split(",") if p]:
        src = item[len("file://"):] if item.startswith("file://") else item
        if not os.path.exists(src):
            raise SubmitError(f"--py-files entry not found: {item}")
        if src.endswith((".zip", ".egg", ".whl")):
            paths.append(os.path.abspath(src))
        else:
            dst = os.path.join(workdir, os.path.basename(src))
            shutil.copy(src, dst)
            if workdir not in paths:
                paths.append(workdir)
    return paths


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("help", "-h", "--help"):
        print(__doc__.strip().split("\n\n")[1])
        return 0 if argv else 1
    try:
        confs, opts, app, app_args = parse_args(argv)
    except SubmitError as e:
        print(f"raydp-submit: {e}", file=sys.stderr)
        return 2
    for w in opts["warnings"]:
        print(f"raydp-submit: warning: {w}", file=sys.stderr)
    from raydp_amd.utils import get_node_ip_address
    ip = get_node_ip_address()
    confs.setdefault("spark.driver.host", ip)
    confs.setdefault("spark.driver.bindAddress", ip)
    confs["spark.master"] = "ray"
    confs.setdefault("spark.app.name", os.path.splitext(os.path.basename(app))[0])
    workdir = tempfile.mkdtemp(prefix="raydp_submit_")
    extra = _stage_py_files(confs.get("spark.submit.pyFiles", ""), workdir)
    app_dir = os.path.dirname(os.path.abspath(app))
    for p in reversed(extra + [app_dir]):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["PYTHONPATH"] = os.pathsep.join(extra + [app_dir] + [os.environ.get("PYTHONPATH", "")]).rstrip(os.pathsep)
    os.environ["RAYDP_SUBMIT_CONF"] = json.dumps(confs)
    if opts["verbose"]:
        print(f"raydp-submit: app={app} args={app_args} confs={confs}", file=sys.stderr)
    import raydp  # noqa: F401  (pyspark / ray facades when those packages are absent)
    from raydp_amd import context, runtime
    runtime.init(**_runtime_kwargs(opts["ray_conf"]))
    old_argv = sys.argv
    sys.argv = [app] + app_args
    rc = 0
    try:
        runpy.run_path(app, run_name="__main__")
    except SystemExit as e:
        rc = int(e.code or 0) if not isinstance(e.code, str) else 1
    finally:
        sys.argv = old_argv
        context.stop_spark()
        runtime.shutdown()
        shutil.rmtree(workdir, ignore_errors=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
