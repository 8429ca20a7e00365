"""raydp-submit (bin/raydp-submit -> raydp_amd.submit): option parsing and end-to-end runs of
a PySpark app on executor processes, including --py-files (reference:
examples/test_raydp_submit_pyfiles.py, test_pyfiles_main.py, test_pyfile.py)."""
import json
import os
import subprocess
import sys

import pytest

from raydp_amd.submit import SubmitError, parse_args

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_args():
    confs, opts, app, args = parse_args(["--ray-conf", "r.json", "--conf", "spark.a=1", "--num-executors", "3",
                                         "--executor-memory=2g", "--py-files", "x.py,y.zip", "--verbose",
                                         "main.py", "--flag", "v"])
    assert confs == {"spark.a": "1", "spark.executor.instances": "3", "spark.executor.memory": "2g",
                     "spark.submit.pyFiles": "x.py,y.zip"}
    assert opts["ray_conf"] == "r.json" and opts["verbose"] and app == "main.py" and args == ["--flag", "v"]
    with pytest.raises(SubmitError):
        parse_args(["--master", "yarn", "a.py"])
    with pytest.raises(SubmitError):
        parse_args(["--class", "org.Foo", "x.jar"])


def test_submit_pi_and_py_files(tmp_path):
    (tmp_path / "helper_mod.py").write_text("def square(x):\n    return x * x\n")
    app = tmp_path / "main_app.py"
    app.write_text(
        "import sys, json\n"
        "from pyspark.sql import SparkSession\n"
        "from helper_mod import square\n"
        "spark = SparkSession.builder.appName('pyfiles').getOrCreate()\n"
        "n = spark.sparkContext.parallelize(range(10), 3).map(square).sum()\n"
        "out = {'n': n, 'execs': spark.conf.get('spark.executor.instances'), 'argv': sys.argv[1:]}\n"
        "open(sys.argv[1], 'w').write(json.dumps(out))\n")
    other = tmp_path / "other"
    other.mkdir()
    result = other / "result.json"
    rc = subprocess.run([os.path.join(ROOT, "bin", "raydp-submit"), "--conf", "spark.executor.instances=2",
                         "--py-files", str(tmp_path / "helper_mod.py"), str(app), str(result)],
                        cwd=str(other), timeout=180).returncode
    assert rc == 0
    out = json.loads(result.read_text())
    assert out["n"] == sum(x * x for x in range(10)) and out["execs"] == "2" and out["argv"] == [str(result)]


_ = sys
