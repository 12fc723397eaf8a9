"""One serving process for every same-model client of a GPU share.

Co-located inference pods that serve the SAME model are not given eight CU
slices and eight copies of the weights: the ledger puts them in one share
group (``sharing.group``), the group's first pod runs this server, and the
others connect to it.  Decode is bound by streaming the weights from HBM, so
one process decoding the clients' combined batch reads them once per step for
everybody: on an MI355X, 8 clients x batch 4 of Llama-3.2-1B decode ~4.9x the
tokens/s of one client alone, against 1.3x as eight separate processes
(reference: "7x GPU density", README.md:31; MPS client bookkeeping,
src/sharing/mig_controller.go:636-678).

Continuous batching over a fixed-shape hipGraph: the decode step is captured
once for ``slots x rows`` batch rows.  A request takes a free slot (a
contiguous group of rows), is prefilled between two graph replays (requests
that wait together and have one prompt length share a prefill pass), decodes
with everyone else, and frees its slot when it has its tokens; unused rows are
parked at position 0.  Tokens are collected on the device and copied out every
``flush`` steps (one sync per flush, not per step).

Wire protocol (Unix socket or TCP, newline-delimited JSON):
  -> {"op": "generate", "prompt": [[int, ...] x rows], "new": n}
  <- {"tokens": [[int, ...] x rows]}      (several, in order)
  <- {"done": true, "new": n, "decode_s": s}
  -> {"op": "stats"}   <- {...}
  -> {"op": "shutdown"}
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import socket
import threading
import time


class _Conn:
    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.out: queue.Queue = queue.Queue()
        self.alive = True
        threading.Thread(target=self._writer, daemon=True).start()

    def send(self, obj: dict) -> None:
        self.out.put(json.dumps(obj).encode() + b"\n")

    def _writer(self) -> None:
        while True:
            b = self.out.get()
            if b is None:
                break
            try:
                self.sock.sendall(b)
            except OSError:
                self.alive = False
                break

    def close(self) -> None:
        self.out.put(None)


class _Slot:
    __slots__ = ("conn", "new", "got", "t_first", "start_step")

    def __init__(self):
        self.conn = None
        self.new = self.got = 0
        self.t_first = 0.0
        self.start_step = 0


class BatchServer:
    """slots x rows decode batch over one model (see the module docstring)."""

    def __init__(self, model, slots: int, rows: int, max_seq: int, flush: int = 16, graph: bool = True):
        import torch

        from ..models.infer import Generator

        self.torch = torch
        self.slots_n, self.rows, self.max_seq, self.flush = slots, rows, max_seq, max(1, flush)
        self.gen = Generator(model, slots * rows, max_seq)
        self.dev = self.gen.dev
        self.vocab = model.cfg.vocab_size
        self.gen.idle_rows(0, slots * rows)
        if self.dev.type == "cuda":
            # Warm the prefill path before the server reports ready: the GEMM library creates
            # its handle and loads its kernels on first use (~170 ms on MI355X), and the decode
            # step of a serving batch runs on kgwe's own kernels, so the first admission would
            # pay for it (time to first token 190-230 ms instead of 13-57 ms).
            warm = torch.zeros(rows, min(32, max_seq - 2), dtype=torch.long, device=self.dev)
            self.gen.prefill(warm, rows=(0, rows))
            self.gen.idle_rows(0, rows)
            torch.cuda.synchronize(self.dev)
        if graph and self.dev.type == "cuda":
            # capture with a valid (parked) state: every row at position 0
            self.gen.capture()
        self.ring = torch.zeros(self.flush, slots * rows, dtype=torch.long, device=self.dev)
        self.host = torch.zeros(self.flush, slots * rows, dtype=torch.long,
                                pin_memory=self.dev.type == "cuda")
        self.slots = [_Slot() for _ in range(slots)]
        self.pending: queue.Queue = queue.Queue()
        self.steps = self.served = self.tokens_out = self.prefill_passes = 0
        self.busy_s = 0.0
        self._stop = threading.Event()
        self._listener: socket.socket | None = None
        self.address = ""

    # ------------------------------------------------------------------ network
    def listen(self, address: str) -> str:
        """address: 'unix:/path/to.sock' or 'host:port' (port 0 = any)."""
        if address.startswith("unix:"):
            path = address[5:]
            try:
                os.unlink(path)
            except FileNotFoundError:
                pass
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            s.bind(path)
            self.address = address
        else:
            host, port = address.rsplit(":", 1)
            s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            s.bind((host, int(port)))
            self.address = f"{host}:{s.getsockname()[1]}"
        s.listen(64)
        self._listener = s
        threading.Thread(target=self._accept, daemon=True).start()
        return self.address

    def _accept(self) -> None:
        while not self._stop.is_set():
            try:
                c, _ = self._listener.accept()
            except OSError:
                return
            threading.Thread(target=self._reader, args=(_Conn(c),), daemon=True).start()

    def _reader(self, conn: _Conn) -> None:
        f = conn.sock.makefile("rb")
        try:
            for line in f:
                try:
                    req = json.loads(line)
                except json.JSONDecodeError:
                    conn.send({"error": "bad json"})
                    continue
                op = req.get("op")
                if op == "generate":
                    err = self._validate(req)
                    if err:
                        conn.send({"error": err})
                    else:
                        self.pending.put((conn, req))
                elif op == "stats":
                    conn.send(self.stats())
                elif op == "shutdown":
                    self._stop.set()
                    self.pending.put(None)
                    conn.send({"ok": True})
                else:
                    conn.send({"error": f"unknown op {op!r}"})
        except OSError:
            pass
        finally:
            conn.alive = False
            conn.close()

    def _validate(self, req: dict) -> str:
        p = req.get("prompt")
        if not isinstance(p, list) or len(p) != self.rows or not all(isinstance(r, list) and r for r in p):
            return f"prompt must be {self.rows} rows of token ids"
        n = len(p[0])
        if any(len(r) != n for r in p):
            return "prompt rows must have one length"
        new = int(req.get("new", 0))
        if new < 1 or n + new + 1 > self.max_seq:
            return f"prompt {n} + new {new} exceeds the server's max sequence {self.max_seq}"
        if any((not isinstance(t, int)) or t < 0 or t >= self.vocab for r in p for t in r):
            return "token id out of range"
        return ""

    def stats(self) -> dict:
        return {"slots": self.slots_n, "rows_per_slot": self.rows, "active": sum(s.conn is not None for s in self.slots),
                "steps": self.steps, "served": self.served, "tokens_out": self.tokens_out,
                "prefill_passes": self.prefill_passes,
                "busy_s": round(self.busy_s, 4), "address": self.address,
                "peak_mem_gb": (self.torch.cuda.max_memory_allocated(self.dev) / 2**30
                                if self.dev.type == "cuda" else 0.0)}

    # ------------------------------------------------------------------ GPU loop
    def _admit_many(self, free: list[int], items: list) -> None:
        """Admit the waiting requests together: those with one prompt length
        that land on consecutive slots share ONE prefill pass (their rows are
        one contiguous range of the batch), so a burst of N same-shape
        requests costs about one prefill of N x rows sequences instead of N
        prefills in a row — the last of 32 waits ~40 ms for its first token
        instead of ~200 ms."""
        torch = self.torch
        by_len: dict[int, list] = {}
        for it in items:
            by_len.setdefault(len(it[1]["prompt"][0]), []).append(it)
        free = sorted(free)
        for group in by_len.values():
            while group:
                run = [free.pop(0)]                      # a run of consecutive free slots
                while free and len(run) < len(group) and free[0] == run[-1] + 1:
                    run.append(free.pop(0))
                batch, group = group[:len(run)], group[len(run):]
                r0, r1 = run[0] * self.rows, (run[-1] + 1) * self.rows
                prompt = torch.tensor([row for _, req in batch for row in req["prompt"]], dtype=torch.long,
                                      device=self.dev)
                self.gen.idle_rows(r0, r1, idle=False)
                first = self.gen.prefill(prompt, rows=(r0, r1)).tolist()
                self.prefill_passes += 1
                now = time.time()
                for j, (idx, (conn, req)) in enumerate(zip(run, batch)):
                    sl = self.slots[idx]
                    sl.conn, sl.new, sl.got = conn, int(req["new"]), 1
                    sl.t_first = now
                    conn.send({"tokens": [[int(t)] for t in first[j * self.rows:(j + 1) * self.rows]]})
                    self.tokens_out += self.rows
                    if sl.got >= sl.new:
                        self._finish(idx)

    def _finish(self, idx: int) -> None:
        sl = self.slots[idx]
        if sl.conn is not None:
            sl.conn.send({"done": True, "new": sl.got, "decode_s": time.time() - sl.t_first})
        self.gen.idle_rows(idx * self.rows, (idx + 1) * self.rows)
        sl.conn = None
        self.served += 1

    def _drain(self, n: int) -> None:
        """Copy the last n steps' tokens out and hand them to their clients."""
        if n == 0:
            return
        torch = self.torch
        self.host[:n].copy_(self.ring[:n], non_blocking=True)
        if self.dev.type == "cuda":
            torch.cuda.current_stream(self.dev).synchronize()
        rows = self.host[:n].tolist()
        for idx, sl in enumerate(self.slots):
            if sl.conn is None:
                continue
            take = min(n, sl.new - sl.got)
            if take <= 0:
                continue
            r0 = idx * self.rows
            if sl.conn.alive:
                sl.conn.send({"tokens": [[rows[t][r0 + r] for t in range(take)] for r in range(self.rows)]})
            sl.got += take
            self.tokens_out += take * self.rows
            if sl.got >= sl.new or not sl.conn.alive:
                self._finish(idx)

    def serve_forever(self) -> None:
        in_ring = 0
        while not self._stop.is_set():
            free = [i for i, s in enumerate(self.slots) if s.conn is None]
            active = self.slots_n - len(free)
            # admit whoever waits (block only when nothing is decoding), all of them together
            if free:
                items = []
                try:
                    item = self.pending.get(block=(active == 0 and in_ring == 0), timeout=0.2)
                    while item is not None:
                        items.append(item)
                        if len(items) >= len(free):
                            break
                        item = self.pending.get_nowait()
                    if item is None and self._stop.is_set():
                        self.pending.put(None)  # the shutdown marker stays for the loop's own check
                except queue.Empty:
                    pass
                if items:
                    self._drain(in_ring)  # tokens of the steps so far belong to the old set of rows
                    in_ring = 0
                    self._admit_many([i for i, s in enumerate(self.slots) if s.conn is None], items)
            if all(s.conn is None for s in self.slots):
                continue
            t0 = time.time()
            # steps until the next slot completes, at most a ring's worth
            left = min(s.new - s.got for s in self.slots if s.conn is not None)
            n = max(1, min(self.flush - in_ring, left - in_ring))
            for _ in range(n):
                self.gen.step(check=False)
                self.ring[in_ring].copy_(self.gen.tok)
                in_ring += 1
                self.steps += 1
            waiting = not self.pending.empty() and any(s.conn is None for s in self.slots)
            if in_ring >= self.flush or in_ring >= left or waiting:
                self._drain(in_ring)
                in_ring = 0
            self.busy_s += time.time() - t0
        self._drain(in_ring)
        if self._listener is not None:
            self._listener.close()

    def stop(self) -> None:
        self._stop.set()
        self.pending.put(None)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kgwe serve-batch")
    ap.add_argument("--model", default="llama3.2-1b")
    ap.add_argument("--slots", type=int, default=8, help="concurrent clients")
    ap.add_argument("--rows", type=int, default=4, help="sequences per client request")
    ap.add_argument("--max-seq", type=int, default=1024)
    ap.add_argument("--flush", type=int, default=16, help="decode steps per token hand-out")
    ap.add_argument("--listen", default=os.environ.get("KGWE_BATCH_ENDPOINT", "127.0.0.1:0"))
    ap.add_argument("--ready-file", default="")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args(argv)
    import torch

    from ..models import llama
    from ..ops import _lib
    from ..utils import sharing

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    share = sharing.apply_from_env(0) if dev.type == "cuda" else sharing.share_info()
    if dev.type == "cuda":
        _lib.lib()
    torch.manual_seed(a.seed)
    model = llama.build(a.model, device=dev, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32)
    model.eval()
    srv = BatchServer(model, a.slots, a.rows, a.max_seq, flush=a.flush, graph=not a.no_graph)
    addr = srv.listen(a.listen)
    print(json.dumps({"listening": addr, "slots": a.slots, "rows": a.rows, "share": share}), flush=True)
    if a.ready_file:
        with open(a.ready_file + ".tmp", "w") as f:
            f.write(addr)
        os.replace(a.ready_file + ".tmp", a.ready_file)
    srv.serve_forever()
    print(json.dumps(srv.stats()), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
