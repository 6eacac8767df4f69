"""bench.py's output contract (the driver parses this line): one JSON object on stdout with the metric,
the whole-job value, the step timing, the run shape, the roofline object of the dominant kernel family,
the BiLSTM roofline and the CPU baseline (the oracle on a bounded sample, port kind), at a small batch
so the test takes seconds. Reference metric: BASELINE.json (text-lines/sec, train step)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env_extra=None):
    env = dict(os.environ)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip().startswith("{")]   # (gloo prints "[Gloo] ..." lines)
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_line_contract():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    d = _run("--steps", "2", "--warmup", "1", "--batch", "32", "--cpu-sample", "2", "--no-sub")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "roofline_lstm", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "bf16"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # whole-job throughput = lines per step / step time
    assert abs(d["value"] - 32 / (d["ms_per_step"] / 1e3)) <= 0.02 * d["value"]
    assert "workload" in d["config"] and "model" not in d["config"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] in ("hbm", "mfma") and r["unit"] in ("GB/s", "TFLOP/s")
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    for part in ("lstm_fwd", "lstm_bwd"):
        lr = d["roofline_lstm"][part]
        assert lr["bound"] == "hbm" and 0 < lr["frac"] < 1
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("port", "reference") and c["value"] > 0 and c["cores"] >= 1


def test_bench_gpus2_spawns_two_ranks():
    """`python bench.py --gpus 2` with no launcher env starts its two ranks itself:
    the line says n_gpus 2, the replicas end bit-identical and the DP overlap fields are there. One-device
    rehearsal: both ranks on cuda:0, gloo over the GPU tensors, per-step BiLSTM launches (the persistent
    sweeps want the whole chip to themselves)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = {"CRNN_SHARE_DEVICE": "1", "CRNN_DIST_BACKEND": "gloo", "CRNN_LSTM_PER_STEP": "1"}
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    d = _run("--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "32", "--no-sub", env_extra=env)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 64
    assert abs(d["value"] - 64 / (d["ms_per_step"] / 1e3)) <= 0.02 * d["value"]
    dp = d["dp"]
    assert dp["param_checksum_spread"] == 0.0
    for k in ("exposed_allreduce_ms_per_step_max_rank", "buckets_per_step", "allreduce_bytes_per_step", "bucket_mb"):
        assert k in dp, k
    assert dp["buckets_per_step"] >= 2 and dp["allreduce_bytes_per_step"] > 0
    assert "cpu_baseline" not in d   # the CPU leg is rank 0 at N = 1 only



def test_bench_gpus2_attaches_configs4_dp_line():
    """An N-rank line also times BASELINE configs[4] in its multi-GPU form (32x1024 crops, 4x768 BiLSTM, batch 64
    per GPU, DP over the same ranks) as sub_measurements.configs4_long_dp, so that the driver's scaling runs observe
    it. One-device rehearsal as above (gloo, per-step BiLSTM launches), one timed step."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = {"CRNN_SHARE_DEVICE": "1", "CRNN_DIST_BACKEND": "gloo", "CRNN_LSTM_PER_STEP": "1"}
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    d = _run("--gpus", "2", "--steps", "1", "--warmup", "1", "--batch", "16", env_extra=env)
    s = d["sub_measurements"]["configs4_long_dp"]
    assert s["n_gpus"] == 2 and s["config"]["parallelism"] == "dp2"
    assert s["config"]["per_gpu_batch"] == 64 and s["config"]["global_batch"] == 128
    assert s["config"]["crop"] == "32x1024" and s["config"]["hidden"] == 768 and s["config"]["rnn_layers"] == 4
    assert s["value"] > 0 and s["dp"]["param_checksum_spread"] == 0.0
