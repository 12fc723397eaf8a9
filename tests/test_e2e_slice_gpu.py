"""Minimum end-to-end slice on one MI355X: a GPUWorkload is
placed by the C++ scheduler (xGMI-aware, RCCL env rendered), the placement is
written as the downward-API annotations file, ``kgwe.launch`` turns it into
the process environment and execs the trainer, which trains on the GPU over
a one-rank RCCL group and writes a sharded checkpoint; a second launch
resumes from it."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_placement_launch_train_resume(tmp_path):
    from kgwe.core import Platform, make_fixture

    plat = Platform({})
    plat.add_fake_node(make_fixture("mi355x-0", 8, 2))
    d = plat.schedule({"metadata": {"name": "slice", "namespace": "ml", "uid": "slice"},
                       "spec": {"gpuRequirements": {"count": 1},
                                "distributedConfig": {"strategy": "FSDP", "worldSize": 1}}})
    assert d["ok"]
    env = dict(d["env"])
    assert env["WORLD_SIZE"] == "1" and env["TORCH_DISTRIBUTED_BACKEND"] == "nccl"
    # Device visibility is the one key this box decides itself (the harness
    # exposes one GPU); everything else comes from the placement.
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        env.pop(k, None)
    env["MASTER_PORT"] = "29517"
    ann = tmp_path / "annotations"
    ann.write_text(f'kgwe.amd.com/rccl-env={json.dumps(json.dumps(env))}\n')
    run_env = dict(os.environ, KGWE_ANNOTATIONS_FILE=str(ann), PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        run_env.pop(k, None)
    ck = tmp_path / "ckpt"
    cmd = [sys.executable, "-m", "kgwe.launch", "--", sys.executable, "-m", "kgwe.bench.train",
           "--model", "tiny", "--seq-len", "256", "--micro-batch", "2", "--ckpt-dir", str(ck)]
    r1 = subprocess.run(cmd + ["--steps", "4"], env=run_env, capture_output=True, text=True,
                        timeout=300, cwd=ROOT)
    assert r1.returncode == 0, r1.stderr[-3000:]
    assert "done at step 4" in r1.stderr
    assert (ck / "latest").read_text() == "step-00000004"
    r2 = subprocess.run(cmd + ["--steps", "6"], env=run_env, capture_output=True, text=True,
                        timeout=300, cwd=ROOT)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert "resumed from" in r2.stderr and "done at step 6" in r2.stderr
