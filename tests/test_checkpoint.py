"""Sharded checkpoint / resume of the data-parallel trainer,
gloo on CPU: an interrupted-and-resumed run matches an uninterrupted one
bit for bit, and a checkpoint written by 2 ranks resumes on 1 (elastic)."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kgwe.bench.train import TrainConfig, Trainer, train
from kgwe.parallel import dist as kdist
from kgwe.parallel.checkpoint import Checkpointer


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg(ckpt_dir, every=0):
    return TrainConfig(model="tiny", seq_len=32, micro_batch=1, parallel="zero",
                       ckpt_dir=ckpt_dir, ckpt_every=every)


def _worker(rank, world, port, ckpt_dir, steps, every, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), KGWE_QUIET="1")
    info = kdist.init(backend="gloo", force_group=True)
    try:
        tr = Trainer(_cfg(ckpt_dir, every), info)
        start = tr.global_step
        train(tr, steps)
        tr.dp.wait_params()
        torch.save({"start": start, "step": tr.global_step,
                    "master": [b.master.clone() for b in tr.dp.buckets]}, f"{out}.rank{rank}")
    finally:
        kdist.shutdown()


def _run(world, ckpt_dir, steps, every, out):
    mp.spawn(_worker, args=(world, _port(), ckpt_dir, steps, every, out), nprocs=world, join=True)
    return [torch.load(f"{out}.rank{r}", weights_only=True) for r in range(world)]


def test_resume_matches_uninterrupted_run(tmp_path):
    full = _run(2, str(tmp_path / "a"), 6, 0, str(tmp_path / "full"))
    part = _run(2, str(tmp_path / "b"), 3, 2, str(tmp_path / "part"))
    assert part[0]["step"] == 3 and (tmp_path / "b" / "latest").read_text() == "step-00000003"
    resumed = _run(2, str(tmp_path / "b"), 6, 0, str(tmp_path / "res"))
    assert resumed[0]["start"] == 3 and resumed[0]["step"] == 6
    for r in range(2):
        for x, y in zip(full[r]["master"], resumed[r]["master"]):
            assert torch.equal(x, y)
    # keep=2: older step directories are pruned
    steps = sorted(p.name for p in (tmp_path / "b").glob("step-*"))
    assert steps == ["step-00000003", "step-00000006"]


def test_elastic_resume_two_ranks_to_one(tmp_path):
    saved = _run(2, str(tmp_path / "c"), 2, 0, str(tmp_path / "two"))
    os.environ.pop("WORLD_SIZE", None)
    os.environ.pop("RANK", None)
    info = kdist.init(backend="gloo", force_group=False)
    tr = Trainer(_cfg(None), info)
    got = Checkpointer(tmp_path / "c").load(tr.dp)
    assert got["step"] == 2 and "gen_state" not in got["extra"]
    for i, b in enumerate(tr.dp.buckets):
        want = torch.cat([saved[0]["master"][i], saved[1]["master"][i]])[:b.numel]
        assert torch.equal(b.master[:b.numel], want)
        # the bf16 weights the model reads were rebuilt from the master
        assert torch.equal(b.flat[:b.numel], want.to(torch.bfloat16))
    if dist.is_initialized():
        dist.destroy_process_group()


def test_load_refuses_shards_of_another_layout_or_step(tmp_path):
    """A shard file that does not belong — truncated tensors, a different
    bucket layout, a rank file copied over another, shards of two different
    steps — is refused, for the same rank count and for the elastic path."""
    _run(2, str(tmp_path / "d"), 2, 0, str(tmp_path / "two"))
    os.environ.pop("WORLD_SIZE", None)
    os.environ.pop("RANK", None)
    info = kdist.init(backend="gloo", force_group=False)
    try:
        tr = Trainer(_cfg(None), info)
        sdir = Checkpointer(tmp_path / "d").latest()
        f0, f1 = sdir / "rank0-of-2.pt", sdir / "rank1-of-2.pt"
        good0 = torch.load(f0, weights_only=True)
        good1 = torch.load(f1, weights_only=True)
        assert Checkpointer(tmp_path / "d").load(tr.dp)["step"] == 2   # intact: loads

        def expect(match):
            with pytest.raises(ValueError, match=match):
                Checkpointer(tmp_path / "d").load(tr.dp)

        bad = {**good1, "buckets": [{k: v[:-64] for k, v in b.items()} for b in good1["buckets"]]}
        torch.save(bad, f1)
        expect("elements")
        torch.save({**good1, "numel": [n + 64 for n in good1["numel"]]}, f1)
        expect("bucket layout")
        torch.save(good0, f1)                      # rank 0's file copied over rank 1's
        expect("file name")
        torch.save({**good1, "step": 7, "dp_step": 7}, f1)
        expect("different steps")
        torch.save(good1, f1)
        # same rank count: a one-rank checkpoint whose tensors were cut short
        one = tmp_path / "e"
        ck = Checkpointer(one)
        ck.save(tr.dp, 5, blocking=True)
        f = ck.latest() / "rank0-of-1.pt"
        p = torch.load(f, weights_only=True)
        torch.save({**p, "buckets": [{k: v[:-64] for k, v in b.items()} for b in p["buckets"]]}, f)
        with pytest.raises(ValueError, match="elements"):
            Checkpointer(one).load(tr.dp)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_checkpoint_side_stream_roundtrip(tmp_path):
    """cuda:0, one process: the pinned side-stream D2H snapshot + background
    write restores exactly the fp32 master / Adam state and the bf16
    weights, and training continues identically."""
    os.environ.pop("WORLD_SIZE", None)
    os.environ.pop("RANK", None)
    info = kdist.init(force_group=False)
    assert info.device.type == "cuda"
    cfg = TrainConfig(model="tiny", seq_len=128, micro_batch=2, parallel="zero")
    ref = Trainer(cfg, info)
    for _ in range(5):
        ref.step()
    ref.dp.wait_params()
    ref_master = [b.master.clone() for b in ref.dp.buckets]
    del ref
    cfg_c = TrainConfig(model="tiny", seq_len=128, micro_batch=2, parallel="zero",
                        ckpt_dir=str(tmp_path), ckpt_every=3)
    a = Trainer(cfg_c, info)
    train(a, 3)
    a.dp.wait_params()
    at3 = [(bb.master.clone(), bb.m.clone(), bb.v.clone(), bb.flat.clone()) for bb in a.dp.buckets]
    del a
    b = Trainer(cfg_c, info)
    assert b.global_step == 3
    b.dp.wait_params()
    for (m0, m1, v1, f1), bb in zip(at3, b.dp.buckets):  # the restore itself is exact
        assert torch.equal(m0, bb.master) and torch.equal(m1, bb.m) and torch.equal(v1, bb.v)
        assert torch.equal(f1, bb.flat)
    train(b, 5)
    b.dp.wait_params()
    # continued training tracks the uninterrupted run (RMSNorm's dw uses fp32
    # atomics, so the two runs differ by summation order only)
    lr = cfg.lr
    for x, y in zip(ref_master, [bb.master for bb in b.dp.buckets]):
        d = (x - y).abs()
        assert d.mean().item() < 0.02 * lr * 5
        assert (d > 0.5 * lr).float().mean().item() < 0.01


@pytest.mark.gpu
def test_gpu_checkpoint_mid_training_holds_one_step(tmp_path):
    """A checkpoint saved while training continues must hold
    exactly the state of its step.  The D2H snapshot runs on a side stream
    and the next steps' AdamW must wait for it (``dp.fence_writes``); the
    step-2 file is compared with a device-side clone taken on the compute
    stream right after step 2, while steps 3-5 run on."""
    os.environ.pop("WORLD_SIZE", None)
    os.environ.pop("RANK", None)
    info = kdist.init(force_group=False)
    assert info.device.type == "cuda"
    cfg = TrainConfig(model="tiny", seq_len=128, micro_batch=2, parallel="zero",
                      ckpt_dir=str(tmp_path), ckpt_every=2)
    a = Trainer(cfg, info)
    a.step()
    a.step()  # global step 2: snapshot launched on a side stream
    a.dp.wait_params()  # compute stream waits for step 2's updates (no host sync)
    want = [(b.master.clone(), b.m.clone(), b.v.clone()) for b in a.dp.buckets]
    for _ in range(3):  # steps 3-5 overwrite master / m / v
        a.step()
    a.ckpt.flush()
    torch.cuda.synchronize()
    payload = torch.load(tmp_path / "step-00000002" / "rank0-of-1.pt", weights_only=True)
    assert payload["step"] == 2
    for (m0, m1, v1), hb in zip(want, payload["buckets"]):
        assert torch.equal(m0.cpu(), hb["master"])
        assert torch.equal(m1.cpu(), hb["m"])
        assert torch.equal(v1.cpu(), hb["v"])
    # and the live state did move on
    assert not torch.equal(want[0][0], a.dp.buckets[0].master)
