"""Submit a PySpark program with raydp-submit (reference: examples/raydp-submit.py).

Writes the runtime description ``ray.conf`` ({"ray": {...}}) that ``raydp-submit --ray-conf``
reads, then runs the Monte-Carlo pi program (examples/pi.py) on one single-core executor.
JVM options of the reference's command line are accepted and ignored (there is no JVM).
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

conf_path = os.path.join(HERE, "ray.conf")
with open(conf_path, "w") as f:
    json.dump({"ray": {"run-mode": "CLUSTER", "num-cpus": 4, "namespace": "raydp-submit-example"}}, f)

java_opts = "-XX:+IgnoreUnrecognizedVMOptions --add-opens=java.base/java.lang=ALL-UNNAMED"
command = [os.path.join(ROOT, "bin", "raydp-submit"), "--ray-conf", conf_path,
           "--conf", "spark.executor.cores=1", "--conf", "spark.executor.instances=1",
           "--conf", "spark.executor.memory=500m",
           "--conf", f"spark.executor.extraJavaOptions={java_opts}",
           "--conf", f"spark.driver.extraJavaOptions={java_opts}",
           "--conf", f"spark.ray.raydp_app_master.extraJavaOptions={java_opts}",
           os.path.join(HERE, "pi.py"), "2"]
sys.exit(subprocess.run(command, check=True).returncode)
