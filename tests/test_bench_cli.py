"""bench.py's launcher contract (CPU: nothing here touches a GPU)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_refuses_fewer_ranks_than_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "one rank per GPU" in r.stderr


def test_bench_parses():
    import ast
    ast.parse(open(os.path.join(REPO, "bench.py")).read())
