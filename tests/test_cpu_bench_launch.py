"""bench.py's launcher guard, on the CPU (no GPU call happens before it): a run whose rank count differs from
--gpus exits non-zero instead of printing a line with the wrong n_gpus."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_refuses_rank_count_mismatch():
    """a launcher that started a different number of ranks than --gpus makes bench.py exit non-zero instead of
    printing a line with the wrong n_gpus"""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"], cwd=REPO,
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "refusing" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.strip().startswith("{")]
