"""Client of kgwe.serving.batch_server: one request, streamed tokens.

A member pod of a share group finds the group's server under
``KGWE_BATCH_ENDPOINT`` (set by the platform with the share's environment).
"""
from __future__ import annotations

import json
import os
import socket
import time


def connect(address: str | None = None, timeout: float = 60.0) -> socket.socket:
    address = address or os.environ.get("KGWE_BATCH_ENDPOINT", "")
    if not address:
        raise ValueError("no batch server address (KGWE_BATCH_ENDPOINT is not set)")
    if address.startswith("unix:"):
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(timeout)
        s.connect(address[5:])
    else:
        host, port = address.rsplit(":", 1)
        s = socket.create_connection((host, int(port)), timeout=timeout)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    return s


def call(address: str | None, obj: dict, timeout: float = 60.0) -> dict:
    with connect(address, timeout) as s:
        s.sendall(json.dumps(obj).encode() + b"\n")
        return json.loads(s.makefile("rb").readline())


def generate(prompt: list, new: int, address: str | None = None, timeout: float = 300.0,
             sock: socket.socket | None = None) -> dict:
    """prompt: rows of token ids (as many rows as the server's --rows).
    Returns {"tokens": rows x new, "t_submit", "t_first", "t_end", "decode_s"}."""
    own = sock is None
    s = sock or connect(address, timeout)
    try:
        t_submit = time.time()
        s.sendall(json.dumps({"op": "generate", "prompt": prompt, "new": new}).encode() + b"\n")
        rows: list[list[int]] = [[] for _ in prompt]
        t_first = 0.0
        for line in s.makefile("rb"):
            msg = json.loads(line)
            if "error" in msg:
                raise RuntimeError(f"batch server: {msg['error']}")
            if "tokens" in msg:
                if not t_first:
                    t_first = time.time()
                for r, t in zip(rows, msg["tokens"]):
                    r.extend(t)
            if msg.get("done"):
                return {"tokens": rows, "t_submit": t_submit, "t_first": t_first, "t_end": time.time(),
                        "decode_s": msg.get("decode_s", 0.0)}
        raise RuntimeError("batch server closed the connection before the request finished")
    finally:
        if own:
            s.close()
