"""Run test_pyfiles_main.py through raydp-submit with --py-files test_pyfile.py
(reference: examples/test_raydp_submit_pyfiles.py)."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def main():
    conf_path = os.path.join(HERE, "ray.conf")
    with open(conf_path, "w") as f:
        json.dump({"ray": {"run-mode": "CLUSTER", "num-cpus": 4}}, f)
    cmd = [os.path.join(ROOT, "bin", "raydp-submit"), "--ray-conf", conf_path,
           "--conf", "spark.executor.cores=1", "--conf", "spark.executor.instances=1",
           "--conf", "spark.executor.memory=500m",
           "--py-files", os.path.join(HERE, "test_pyfile.py"), os.path.join(HERE, "test_pyfiles_main.py")]
    # run from elsewhere so only --py-files can make test_pyfile importable
    return subprocess.run(cmd, cwd="/", check=False).returncode


if __name__ == "__main__":
    sys.exit(main())
