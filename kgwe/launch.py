"""Container entrypoint wrapper: export the placement the extender bound.

The extender writes the placement to pod annotations at bind time
(kgwe.amd.com/rccl-env etc.); the controller mounts them through the
downward API at /etc/kgwe/annotations.  `python -m kgwe.launch -- <cmd>`
parses that file, exports HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES, the
RCCL rendezvous (MASTER_ADDR/PORT, WORLD_SIZE, NPROC_PER_NODE) and NCCL_*
tuning, then replaces itself with <cmd> (typically torchrun).  It execs
BEFORE anything touches the GPU, so the exec is safe.

A co-located share's HBM cap (KGWE_GPU_MEMORY_FRACTION) is enforced, not just
exported: the launcher puts ``kgwe/_sitehook`` first on PYTHONPATH, whose
``sitecustomize`` caps PyTorch's allocator in every Python process of the
workload as soon as that process imports torch.
"""
from __future__ import annotations

import json
import os
import sys

ANN_FILE = os.environ.get("KGWE_ANNOTATIONS_FILE", "/etc/kgwe/annotations")
ANN_ENV = "kgwe.amd.com/rccl-env"
SITEHOOK = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_sitehook")


def enforce_share_limits(env: dict) -> dict:
    """With an HBM cap in the placement, make every Python process of the
    workload install it at start-up (see kgwe/_sitehook/sitecustomize.py)."""
    try:
        frac = float(env.get("KGWE_GPU_MEMORY_FRACTION", "0") or 0)
    except ValueError:
        frac = 0.0
    if 0.0 < frac < 1.0:
        parts = [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p and p != SITEHOOK]
        env["PYTHONPATH"] = os.pathsep.join([SITEHOOK] + parts)
    return env


def parse_downward_api(text: str) -> dict:
    """Downward API annotation file: one `key="json-escaped value"` per line."""
    out = {}
    for line in text.splitlines():
        if "=" not in line:
            continue
        k, v = line.split("=", 1)
        v = v.strip()
        if v.startswith('"'):
            try:
                v = json.loads(v)
            except json.JSONDecodeError:
                v = v.strip('"')
        out[k.strip()] = v
    return out


def placement_env(annotations: dict) -> dict:
    env = json.loads(annotations.get(ANN_ENV, "{}") or "{}")
    return {str(k): str(v) for k, v in env.items()}


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] == "--":
        argv = argv[1:]
    if not argv:
        print("usage: python -m kgwe.launch -- <command> [args...]", file=sys.stderr)
        return 2
    env = dict(os.environ)
    try:
        with open(ANN_FILE) as f:
            env.update(placement_env(parse_downward_api(f.read())))
    except FileNotFoundError:
        print(f"[kgwe.launch] {ANN_FILE} not found: running without a kgwe placement",
              file=sys.stderr)
    enforce_share_limits(env)
    os.execvpe(argv[0], argv, env)
    return 127  # not reached


if __name__ == "__main__":
    raise SystemExit(main())
