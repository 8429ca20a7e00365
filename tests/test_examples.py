"""The ported examples run end to end on CPU (reference: examples/*.py)."""
import os
import subprocess
import sys

import pytest

EX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")


@pytest.mark.parametrize("script,args,expect", [
    ("pytorch_nyctaxi.py", [], "_training_iteration"),
    ("raytrain_nyctaxi.py", [], "final"),
    ("horovod_nyctaxi.py", ["--epochs", "1"], "'epoch': 1"),
    ("xgboost_ray_nyctaxi.py", [], "Final validation rmse"),
    ("raydp-submit.py", [], "Pi is roughly"),
    ("tensorflow_nyctaxi.py", [], "TensorFlow is not installed"),
    ("test_raydp_submit_pyfiles.py", [], "py-files OK"),
    ("random_nyctaxi.py", ["--num-records", "1000", "--output", "/tmp/raydp_random_nyctaxi.csv"], "wrote 1000 rows"),
])
def test_example_runs(script, args, expect):
    env = dict(os.environ, NYC_EPOCHS="1")
    r = subprocess.run([sys.executable, os.path.join(EX, script)] + args, cwd=EX, env=env, timeout=400,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert r.returncode == 0, r.stdout[-3000:]
    assert expect in r.stdout, r.stdout[-3000:]


def test_raytrain_tutorial_runs():
    """tutorials/raytrain_example.ipynb port (B4 workload): legacy Trainer + to_torch shards."""
    tut = os.path.join(os.path.dirname(EX), "tutorials", "raytrain_example.py")
    env = dict(os.environ, RAYTRAIN_EPOCHS="2")
    r = subprocess.run([sys.executable, tut], cwd=os.path.dirname(tut), env=env, timeout=400,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "test_acc" in r.stdout and "'epoch': 1" in r.stdout, r.stdout[-3000:]
