"""bench.py's driver contract, run as the driver runs it: one JSON line from rank 0 with the
BASELINE metric, and -- before the 8-GPU node ever sees it -- the torchrun data-parallel path
(one process per rank, barrier + max-over-ranks timing, per-layer gradient buckets on a
communication stream).  On the one-GPU box the two ranks share the card and talk over gloo;
the node run uses the same code with --backend nccl (RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, timeout=240):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _common(res, n, workload):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in res, k
    assert res["n_gpus"] == n and res["config"]["parallelism"] == f"dp{n}"
    assert res["value"] > 0 and res["scaling"] == "weak" and res["higher_is_better"] is True
    assert res["config"]["workload"].startswith(workload)
    assert res["roofline"]["bound"] == "mfma" and 0 < res["roofline"]["frac"] < 1
    assert res["fp16_overflow_steps"] == 0


def test_torchrun_two_ranks_gloo():
    res = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                "--backend", "gloo", "--steps", "2", "--warmup", "1", "--coords", "65536", "--hidden", "256",
                "--layers", "3", "--no-cpu-baseline"])
    _common(res, 2, "cfg2")
    assert res["config"]["global_batch"] == 2 * 65536 and res["config"]["backend"] == "gloo"
    assert "cpu_baseline" not in res and "recon_snr" not in res
    # what the process group saw, and how much of the all-reduce the backward hid
    d = res["dist"]
    assert d["backend"] == "gloo" and d["world_size_seen"] == 2 and d["rccl"] is False
    assert d["bucketed_overlap"] is True and d["buckets"] == 2 + 2  # head, 2 inner layers, first layer
    assert d["ms_per_step_with_allreduce"] > 0 and d["ms_per_step_without_allreduce"] > 0
    assert d["allreduce_alone_ms"] > 0
    assert abs(d["exposed_allreduce_ms_per_step"]
               - (d["ms_per_step_with_allreduce"] - d["ms_per_step_without_allreduce"])) < 1e-9


def test_single_gpu_line_carries_recon_snr():
    """The default line carries both halves of BASELINE's metric: coord-samples/s and, outside the
    timed region, the recon SNR of the headline model's fit against the reference's run of it."""
    res = _run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--coords", "65536",
                "--no-cpu-baseline"])
    r = res["recon_snr"]
    assert r is not None and r["fixture"].startswith("tests/golden/")
    assert abs(r["snr_target_db"] - r["reference_snr_target_db"]) < r["tolerance_db"], r
    assert r["fp16_overflow_steps"] == 0 and r["final_lr"] == r["reference_final_lr"]
    assert "dist" not in res


def test_torchrun_two_ranks_strong_scaling():
    """--strong: the global batch is fixed and split over the ranks (SURVEY §8e's strong curve)."""
    res = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                "--backend", "gloo", "--steps", "2", "--warmup", "1", "--coords", "131072", "--hidden", "256",
                "--layers", "3", "--strong", "--no-cpu-baseline"])
    assert res["n_gpus"] == 2 and res["scaling"] == "strong" and res["value"] > 0
    assert res["config"]["global_batch"] == 131072 and res["config"]["coords_per_gpu"] == 65536


def test_kan_config():
    res = _run([sys.executable, "bench.py", "--config", "cfg5", "--steps", "2", "--warmup", "1", "--coords", "50000"])
    assert res["n_gpus"] == 1 and res["value"] > 0 and res["dtype"] == "fp32"
    assert res["config"]["widths"] == [1, 64, 64, 1] and res["roofline"]["bound"] == "mfma"
    assert 0 < res["roofline"]["frac"] < 1 and res["roofline"]["kernel"].startswith("kan_")


@pytest.mark.parametrize("cfg,extra", [("cfg3", ["--coords", "262144"]), ("cfg4", [])])
def test_single_gpu_configs(cfg, extra):
    res = _run([sys.executable, "bench.py", "--config", cfg, "--steps", "2", "--warmup", "1",
                "--no-cpu-baseline", *extra])
    _common(res, 1, cfg)
    assert res["config"]["in_features"] == 2
    assert res["config"]["layers"] == (6 if cfg == "cfg3" else 5)
