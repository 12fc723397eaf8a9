"""Sharded checkpoint / resume for the data-parallel trainer (the reference keeps all state in process memory; its example mounts a
checkpoint PVC for the user job, examples/distributed-training.yaml:80-90).

What a rescheduled workload (controller ``spec.recovery``) resumes from:

* every rank writes ITS optimizer shard (fp32 master, Adam m / v per bucket —
  the bf16 weights are derived from the master) plus the step counter and
  its data-generator state: ``<dir>/step-<N>/rank<r>-of-<W>.pt``;
* the device -> host copy runs on a side HIP stream into pinned buffers and
  the file is written by a background thread, so a checkpoint costs the
  training loop one stream hand-off, not the write; the step directory is
  published (``<dir>/latest``) by rank 0 only after every rank has finished
  (barrier), so a crash mid-write never leaves a torn "latest";
* resume is elastic: shards written by W ranks are re-sliced for the W' ranks
  that load them (a job rescheduled onto a different GPU count keeps its
  optimizer state); files are read with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch
import torch.distributed as dist


def _dist_info():
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class Checkpointer:
    def __init__(self, directory: str | os.PathLike, keep: int = 2):
        self.dir = Path(directory)
        self.keep = keep
        self._thread: threading.Thread | None = None
        self._error: BaseException | None = None
        self._pending: Path | None = None  # written, not yet published
        self._host: list[dict] | None = None  # pinned snapshot buffers, reused across saves

    # ------------------------------------------------------------------ save
    def save(self, dp, step: int, extra: dict | None = None, blocking: bool = False) -> Path:
        """Snapshot ``dp`` (a ShardedDataParallel) at ``step``.  Returns the
        step directory; the write completes in the background unless
        ``blocking`` (call ``wait()`` before the next save / exit)."""
        self.flush()  # publish the previous step: its write had a whole interval
        rank, world = _dist_info()
        sdir = self.dir / f"step-{step:08d}"
        sdir.mkdir(parents=True, exist_ok=True)
        dp.wait_params()
        state = dp.shard_state()
        cuda = dp.device.type == "cuda"
        stream = torch.cuda.Stream(dp.device) if cuda else None
        host = []
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream(dp.device))
        # flush() above joined the previous write, so its buffers are free again
        reuse = self._host if self._host is not None and len(self._host) == len(state["buckets"]) \
            and all(hb[k].shape == t.shape for hb, b in zip(self._host, state["buckets"])
                    for k, t in b.items()) else None
        with torch.cuda.stream(stream) if stream is not None else _null():
            for i, b in enumerate(state["buckets"]):
                hb = {}
                for k, t in b.items():
                    h = reuse[i][k] if reuse is not None else torch.empty(
                        t.shape, dtype=t.dtype, pin_memory=cuda)
                    h.copy_(t, non_blocking=cuda)
                    hb[k] = h
                host.append(hb)
        self._host = host
        done = torch.cuda.Event() if cuda else None
        if done is not None:
            done.record(stream)
            # the next step's AdamW (side stream or compute stream) must not
            # overwrite master / m / v while this copy still reads them
            dp.fence_writes(done)
        payload = {"step": int(step), "dp_step": state["step"], "world": world, "rank": rank,
                   "numel": [b.numel for b in dp.buckets], "buckets": host, "extra": extra or {}}
        path = sdir / f"rank{rank}-of-{world}.pt"

        def write():
            try:
                if done is not None:
                    done.synchronize()
                tmp = path.with_suffix(".tmp")
                torch.save(payload, tmp)
                os.replace(tmp, path)
            except BaseException as e:  # noqa: BLE001 - surfaced by wait()
                self._error = e

        self._thread = threading.Thread(target=write, name="kgwe-ckpt", daemon=True)
        self._thread.start()
        self._pending = sdir
        if blocking:
            self.flush()
        return sdir

    def flush(self) -> None:
        """Finish the in-flight write (all ranks) and publish it."""
        if self._pending is not None:
            sdir, self._pending = self._pending, None
            self.publish(sdir)
        else:
            self.wait()

    def wait(self) -> None:
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise RuntimeError(f"checkpoint write failed: {e}") from e

    def publish(self, sdir: Path) -> None:
        """Every rank's file is on disk (barrier) -> rank 0 points ``latest``
        at the step and prunes old steps."""
        self.wait()
        if dist.is_initialized():
            dist.barrier()
        rank, _ = _dist_info()
        if rank == 0:
            tmp = self.dir / "latest.tmp"
            tmp.write_text(sdir.name)
            os.replace(tmp, self.dir / "latest")
            steps = sorted(p for p in self.dir.glob("step-*") if p.is_dir())
            for old in steps[:-self.keep]:
                for f in old.iterdir():
                    f.unlink()
                old.rmdir()
        if dist.is_initialized():
            dist.barrier()

    # ------------------------------------------------------------------ load
    def latest(self) -> Path | None:
        marker = self.dir / "latest"
        if not marker.exists():
            return None
        sdir = self.dir / marker.read_text().strip()
        return sdir if sdir.is_dir() else None

    @torch.no_grad()
    def load(self, dp, sdir: Path | None = None) -> dict | None:
        """Restore ``dp`` from the latest (or given) step; returns the saved
        ``{"step", "extra"}`` or None when there is no checkpoint."""
        sdir = sdir or self.latest()
        if sdir is None:
            return None
        rank, world = _dist_info()
        files = sorted(sdir.glob("rank*-of-*.pt"))
        if not files:
            return None
        saved_world = int(files[0].name.split("-of-")[1].split(".")[0])
        if saved_world == world:
            payload = torch.load(sdir / f"rank{rank}-of-{world}.pt", weights_only=True)
            _check_layout(payload, dp, world, rank)
            state = {"step": payload["dp_step"], "world": world, "rank": rank,
                     "buckets": payload["buckets"]}
        else:  # elastic: re-slice every saved shard for this rank
            parts = [torch.load(sdir / f"rank{r}-of-{saved_world}.pt", weights_only=True)
                     for r in range(saved_world)]
            payload = parts[0]
            for r, part in enumerate(parts):  # every saved shard belongs to this model and to one step
                _check_layout(part, dp, saved_world, r)
                if part["dp_step"] != payload["dp_step"] or int(part["step"]) != int(payload["step"]):
                    raise ValueError(f"checkpoint shards of different steps in {sdir} "
                                     f"(rank 0: {payload['step']}, rank {r}: {part['step']})")
            buckets = []
            for i, b in enumerate(dp.buckets):
                lo = rank * b.shard
                nb = {}
                for k in ("master", "m", "v"):
                    full = torch.cat([p["buckets"][i][k] for p in parts])[:b.numel]
                    sl = torch.zeros(b.shard, dtype=full.dtype)
                    hi = min(b.numel, lo + b.shard)
                    if hi > lo:
                        sl[:hi - lo] = full[lo:hi]
                    nb[k] = sl
                buckets.append(nb)
            state = {"step": payload["dp_step"], "world": world, "rank": rank, "buckets": buckets}
            # per-rank data-generator states do not carry over to a new rank count
            payload = {**payload, "extra": {k: v for k, v in (payload.get("extra") or {}).items()
                                            if k != "gen_state"}}
        dev = dp.device
        state["buckets"] = [{k: t.to(dev) for k, t in b.items()} for b in state["buckets"]]
        dp.load_shard_state(state)
        return {"step": int(payload["step"]), "extra": payload.get("extra") or {}}


def _check_layout(payload: dict, dp, world: int, rank: int) -> None:
    """A saved shard must come from this model's bucket layout: same bucket
    sizes, the rank / world its file name says, and shards of the length that
    world implies (a stale or foreign file would otherwise be sliced into the
    optimizer state silently)."""
    numel = [b.numel for b in dp.buckets]
    if list(payload.get("numel", [])) != numel:
        raise ValueError("checkpoint bucket layout does not match this model "
                         f"(saved {list(payload.get('numel', []))[:4]}..., model {numel[:4]}...)")
    if int(payload.get("world", world)) != world or int(payload.get("rank", rank)) != rank:
        raise ValueError(f"checkpoint shard says rank {payload.get('rank')} of {payload.get('world')}, "
                         f"its file name rank {rank} of {world}")
    if len(payload["buckets"]) != len(numel):
        raise ValueError("checkpoint has a different number of buckets than this model")
    for i, (n, saved) in enumerate(zip(numel, payload["buckets"])):
        align = world * 64
        shard = -(-n // align) * align // world
        for k in ("master", "m", "v"):
            if k not in saved or saved[k].numel() != shard:
                raise ValueError(f"checkpoint bucket {i} '{k}' has {saved[k].numel() if k in saved else 0} "
                                 f"elements, a {world}-rank shard of {n} has {shard}")


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
