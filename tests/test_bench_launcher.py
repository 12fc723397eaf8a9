"""bench.py as the driver runs it: ``python bench.py --gpus N`` with no
WORLD_SIZE spawns N rank processes (torch.distributed.run, child process) and
re-emits rank 0's JSON line.  CPU: gloo ranks on a tiny model; GPU: one rank
through the same launcher."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(gpus: int, extra: list[str], timeout: int = 300, env_extra: dict | None = None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    cmd = [sys.executable, "bench.py", "--gpus", str(gpus), "--steps", "2", "--warmup", "1",
           "--no-sched", "--no-cluster", "--no-busbw", *extra]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    return r, lines


def test_bench_gpus2_spawns_two_gloo_ranks():
    r, lines = _run(2, ["--model", "tiny", "--seq-len", "64", "--micro-batch", "2",
                        "--fsdp-row", "on"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, lines  # exactly one JSON line on stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == "zero2-dp2"
    assert out["config"]["global_batch"] == 4
    assert "torch.distributed.run" in out["launcher"]
    l0, l1 = out["loss_per_rank"]
    assert l0 != l1  # the two ranks trained on different synthetic batches
    assert out["fsdp_row"]["parallelism"] == "fsdp2"
    assert out["fsdp_row"]["tokens_per_s"] > 0
    assert out["tokens_per_s"] > 0 and out["ms_per_step"] > 0
    # the launcher's per-link xGMI probe ran (a CPU host has no GPUs to probe)
    assert "xgmi_probe" in out and out["xgmi_probe"].get("devices", 0) < 2


def test_bench_gpus4_rehearses_the_multi_rank_path():
    """Four gloo ranks through the same launcher (the driver's N=4 point): the
    sharded-DP headline row and the FSDP2 row both run and every rank
    reports (the busBW sweep is off: 1 GiB all-reduces on gloo)."""
    r, lines = _run(4, ["--model", "tiny", "--seq-len", "64", "--micro-batch", "1",
                        "--fsdp-row", "on", "--reduce-row", "on"], timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(lines[-1])
    assert out["n_gpus"] == 4 and out["config"]["parallelism"] == "zero2-dp4"
    assert out["config"]["global_batch"] == 4
    assert len(out["loss_per_rank"]) == 4 and len(set(out["loss_per_rank"])) == 4
    assert out["fsdp_row"]["parallelism"] == "fsdp4" and "error" not in out["fsdp_row"]
    assert out["config"]["grad_reduce_dtype"] == "bf16"
    rr = out["reduce_dtype_row"]  # the fp32-reduce row ran (or says why not)
    assert rr.get("grad_reduce_dtype") == "fp32" or "error" in rr, rr


def test_bench_gpus8_rehearses_the_drivers_headline_point():
    """Eight gloo ranks (the driver's N=8 point, the BASELINE config's rank
    count): headline row, reduce-dtype row and FSDP2 row all run, every rank
    reports its own loss, and the job-wide token rate is the sum over ranks."""
    r, lines = _run(8, ["--model", "tiny", "--seq-len", "64", "--micro-batch", "1",
                        "--fsdp-row", "on", "--reduce-row", "on"], timeout=600,
                    env_extra={"OMP_NUM_THREADS": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, lines
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "zero2-dp8"
    assert out["config"]["global_batch"] == 8 and out["scaling"] == "weak"
    assert len(out["loss_per_rank"]) == 8 and len(set(out["loss_per_rank"])) == 8
    assert len(out["util_per_rank"]) == 8
    assert out["fsdp_row"]["parallelism"] == "fsdp8" and "error" not in out["fsdp_row"]
    rr = out["reduce_dtype_row"]
    assert rr.get("grad_reduce_dtype") == "fp32" or "error" in rr, rr
    # whole-job rate: 8 ranks x 64 tokens per step
    assert abs(out["tokens_per_s"] - 8 * 64 / (out["ms_per_step"] / 1e3)) < 0.02 * out["tokens_per_s"]
    assert abs(out["tokens_per_s_per_gpu"] * 8 - out["tokens_per_s"]) < 0.02 * out["tokens_per_s"]


def test_bench_failing_rank_fails_the_launcher():
    # An impossible model name makes every rank raise: the launcher must exit
    # non-zero and print no result line.
    r, lines = _run(2, ["--model", "no-such-model"], timeout=200)
    assert r.returncode != 0
    assert not any(ln.startswith('{"metric"') for ln in lines)


def test_bench_rank_refuses_mismatched_world():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1"}
    r, lines = _run(2, ["--model", "tiny", "--seq-len", "64"], env_extra=env, timeout=200)
    assert r.returncode == 2
    assert not any(ln.startswith('{"metric"') for ln in lines)


@pytest.mark.gpu
def test_bench_gpus1_through_launcher_on_gpu():
    # amd-smi's gfx_activity is a smoothed busy % (it needs up to ~1 s of load
    # to rise on some hosts): time enough steps for it to settle.
    r, lines = _run(1, ["--model", "llama3-8b", "--seq-len", "2048", "--micro-batch", "1",
                        "--steps", "24", "--warmup", "4"], timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(lines[-1])
    assert out["n_gpus"] == 1 and "torch.distributed.run" in out["launcher"]
    assert out["attention"] == "kgwe_flash_attn"
    assert out["steps"] == 24
    assert out["value"] is not None and out["value"] > 50.0
    assert out["util_whole_process_pct"] is not None


def test_stuck_secondary_rows_cannot_cost_the_headline():
    """The rows after the headline run under a watchdog at N > 1.  With a limit
    no row can meet, rank 0 still prints exactly one line, the measured
    headline intact and the unfinished rows marked, and the job exits 0."""
    r, lines = _run(2, ["--model", "tiny", "--seq-len", "64", "--micro-batch", "2", "--fsdp-row", "on",
                        "--reduce-row", "on", "--extra-rows-timeout", "0.01"], timeout=200)
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, lines
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ms_per_step"] > 0 and out["tokens_per_s"] > 0
    assert len(out["loss_per_rank"]) == 2
    assert "watchdog" in out["fsdp_row"]["error"]
    assert "watchdog" in out["reduce_dtype_row"]["error"] or out["reduce_dtype_row"].get("grad_reduce_dtype")
    assert "secondary rows timed out" in r.stderr
