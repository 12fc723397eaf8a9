"""bf16 decode throughput, alone and as co-located clients of ONE GPU
(BASELINE.json config 4: "one GPU split 8-way, 8 bf16 inference pods";
reference README.md:31 "7x GPU density").

``run``       one decode client: build a random-init Llama (bf16), prefill a
              synthetic prompt, capture the decode step in a hipGraph, then
              time ``--new`` greedy decode steps.  Prints one JSON line.
``client``    one client of a share group's batch server (no GPU in this
              process): waits for the go file, sends its prompt, streams tokens.
``colocate``  the platform path end to end on the local GPU: the C++
              scheduler ledger places ``--clients`` CoLocate shares on the
              GPU (``Platform.schedule`` of GPUWorkload-shaped requests ->
              disjoint HSA_CU_MASK ranges + HBM caps), then one ``run``
              process per share is started with exactly the env the pod
              would get (``kgwe.launch`` semantics).  All clients start
              decoding at the same instant; reported: per-client and
              aggregate tokens/s, against (a) one client alone on the whole
              GPU and (b) one process decoding the clients' combined batch.
              The parent never touches the GPU (no HIP call): it only spawns.
              ``--share-mode batched``: the clients are ONE share group — the
              ledger gives the group one CU range and one HBM cap, the leader's
              env starts ``kgwe.serving.batch_server`` (weights once, continuous
              batching), and every client talks to it over the group's socket.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


# --------------------------------------------------------------------------- client
def run_client(a) -> dict:
    import torch

    from ..models import llama
    from ..models.infer import Generator
    from ..ops import _lib
    from ..utils import sharing

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    share = sharing.apply_from_env(0) if dev.type == "cuda" else sharing.share_info()
    if dev.type == "cuda":
        _lib.lib()  # the HIP kernels must load on a GPU host
    torch.manual_seed(a.seed)
    t0 = time.time()
    model = llama.build(a.model, device=dev, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32)
    model.eval()
    cfg = model.cfg
    gen = Generator(model, a.batch, a.prompt + a.new + 1)
    prompt = torch.randint(0, cfg.vocab_size, (a.batch, a.prompt), device=dev)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    t_pf = time.time()
    gen.prefill(prompt)
    sync()
    ttft = time.time() - t_pf
    if not a.no_graph:
        gen.capture()
    for _ in range(a.warmup):  # graph replays warm clocks / caches; rewound below
        gen.step()
    sync()
    gen.prefill(prompt)  # same prompt: cache positions rewritten, positions reset
    sync()
    build_s = time.time() - t0
    if a.ready_file:
        open(a.ready_file, "w").close()
        while not os.path.exists(a.go_file):
            time.sleep(0.005)
        go = float(open(a.go_file).read().strip() or 0)
        while time.time() < go:
            pass
    ts = time.time()
    for _ in range(a.new - 1):
        gen.step()
    sync()
    te = time.time()
    toks = a.batch * (a.new - 1)
    return {"model": a.model, "batch": a.batch, "prompt": a.prompt, "new_tokens": a.new,
            "graph": not a.no_graph, "tokens": toks, "t_start": ts, "t_end": te,
            "decode_s": te - ts, "tokens_per_s": toks / (te - ts), "step_ms": 1000 * (te - ts) / (a.new - 1),
            "ttft_s": ttft, "build_s": build_s, "share": share,
            "peak_mem_gb": (torch.cuda.max_memory_allocated(dev) / 2**30 if dev.type == "cuda" else 0.0),
            "last_tokens": gen.tok[:4].tolist()}


def run_group_client(a) -> dict:
    """A member of a share group: tokens come from the group's server."""
    import random

    from ..serving import client

    rnd = random.Random(a.seed)
    prompt = [[rnd.randrange(0, a.vocab) for _ in range(a.prompt)] for _ in range(a.batch)]
    sock = client.connect(a.endpoint or None, timeout=a.timeout)
    if a.ready_file:
        open(a.ready_file, "w").close()
        while not os.path.exists(a.go_file):
            time.sleep(0.005)
        go = float(open(a.go_file).read().strip() or 0)
        while time.time() < go:
            pass
    r = client.generate(prompt, a.new, sock=sock, timeout=a.timeout)
    sock.close()
    toks = a.batch * (a.new - 1)  # the tokens after the prefill's, as run_client counts them
    dt = r["t_end"] - r["t_first"]
    return {"batch": a.batch, "prompt": a.prompt, "new_tokens": a.new, "tokens": toks,
            "t_submit": r["t_submit"], "t_start": r["t_first"], "t_end": r["t_end"], "decode_s": dt,
            "tokens_per_s": toks / dt, "step_ms": 1000 * dt / (a.new - 1),
            "ttft_s": r["t_first"] - r["t_submit"], "last_tokens": [row[-1] for row in r["tokens"]][:4]}


# --------------------------------------------------------------------------- parent
def _client_cmd(a, batch: int) -> list[str]:
    return [sys.executable, "-m", "kgwe.bench.infer", "run", "--model", a.model, "--batch", str(batch),
            "--prompt", str(a.prompt), "--new", str(a.new), "--warmup", str(a.warmup), "--json"] + \
        (["--no-graph"] if a.no_graph else [])


def _run_alone(a, batch: int, env: dict | None = None) -> dict:
    r = subprocess.run(_client_cmd(a, batch), cwd=ROOT, capture_output=True, text=True,
                       timeout=a.timeout, env=env or dict(os.environ))
    js = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not js:
        raise RuntimeError(f"client failed rc={r.returncode}: {r.stderr[-1500:]}")
    return json.loads(js[-1])


def place_shares(n: int, cu_percent: float, memory_gb: float, group: str = "",
                 socket_dir: str = "") -> tuple[list[dict], str]:
    """Shares from the real scheduler ledger: the local GPU via amd-smi when
    present (else a mocked MI355X node).  group: all n are one share group."""
    from ..core import Platform, amdsmi_discover, make_fixture

    p = Platform(dict({"enforceBudgets": False}, **({"shareSocketDir": socket_dir} if socket_dir else {})))
    src = "amd-smi"
    d = amdsmi_discover("local")
    if d.get("ok") and (d.get("node") or {}).get("gpus"):
        p.add_amdsmi_node("local")
    else:
        p.add_fake_node(make_fixture("local", 8, 2))
        src = "fixture"
    out = []
    for i in range(n):
        w = {"metadata": {"name": f"serve-{i}", "namespace": "inference", "uid": f"serve-{i}"},
             "spec": {"workloadType": "Inference",
                      "gpuRequirements": {"count": 1, "sharing": {"method": "CoLocate",
                                                                   "cuPercent": cu_percent,
                                                                   "memoryGB": memory_gb}}}}
        if group:
            w["spec"]["gpuRequirements"]["sharing"]["group"] = group
        dd = p.schedule(w)
        if not dd.get("ok"):
            raise RuntimeError(f"share {i} not placed: {dd.get('failed_nodes')}")
        out.append(dd)
    return out, src


def _wait_ready(paths: list[str], procs: list, deadline: float, what: str) -> None:
    while not all(os.path.exists(p) for p in paths):
        if time.time() > deadline or any(p.poll() not in (None, 0) for p in procs):
            for p in procs:
                p.kill()
            errs = [p.communicate()[1][-800:] for p in procs if p.returncode not in (None, 0)]
            raise RuntimeError(f"{what} did not get ready: {errs[:2]}")
        time.sleep(0.05)


def colocate_batched(a) -> dict:
    """--share-mode batched: one share group, one serving process."""
    from ..models import llama

    tmp = tempfile.mkdtemp(prefix="kgwe-group-")
    shares, src = place_shares(a.clients, a.cu_percent, a.memory_gb, group=a.model, socket_dir=tmp)
    lead = [s for s in shares if s.get("share_leader")]
    assert len(lead) == 1 and all(s["shared_gpu"] == lead[0]["shared_gpu"] for s in shares), shares
    endpoint = lead[0]["env"]["KGWE_BATCH_ENDPOINT"]
    res: dict = {"mode": "batched", "clients": a.clients, "model": a.model, "batch_per_client": a.batch,
                 "prompt": a.prompt, "new_tokens": a.new, "topology_source": src,
                 "shared_gpus": sorted({s["shared_gpu"] for s in shares}),
                 "cu_masks": sorted({s["env"]["HSA_CU_MASK"] for s in shares}),
                 "roles": [s["env"]["KGWE_SHARE_ROLE"] for s in shares],
                 "hbm_cap": lead[0]["env"].get("KGWE_GPU_MEMORY_FRACTION")}
    if not a.skip_baselines:
        res["alone"] = _run_alone(a, a.batch)
    env = dict(os.environ)
    env.update(lead[0]["env"])
    env["HIP_VISIBLE_DEVICES"] = env["ROCR_VISIBLE_DEVICES"] = "0"
    from ..launch import enforce_share_limits

    enforce_share_limits(env)  # what `python -m kgwe.launch` does in the pod
    server = subprocess.Popen(
        [sys.executable, "-m", "kgwe.serving.batch_server", "--model", a.model, "--slots", str(a.clients),
         "--rows", str(a.batch), "--max-seq", str(a.prompt + a.new + 1), "--flush", str(a.flush),
         "--ready-file", f"{tmp}/server-ready"],
        cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    deadline = time.time() + a.timeout
    try:
        _wait_ready([f"{tmp}/server-ready"], [server], deadline, "batch server")
        vocab = llama.PRESETS[a.model].vocab_size
        procs = []
        for i, s in enumerate(shares):
            cenv = dict(os.environ)
            cenv.update({k: v for k, v in s["env"].items() if k.startswith("KGWE_")})
            cenv["HIP_VISIBLE_DEVICES"] = cenv["ROCR_VISIBLE_DEVICES"] = ""  # a member never opens the GPU
            cmd = [sys.executable, "-m", "kgwe.bench.infer", "client", "--batch", str(a.batch),
                   "--prompt", str(a.prompt), "--new", str(a.new), "--seed", str(a.seed + i), "--vocab", str(vocab),
                   "--endpoint", endpoint, "--ready-file", f"{tmp}/ready{i}", "--go-file", f"{tmp}/go",
                   "--timeout", str(a.timeout), "--json"]
            procs.append(subprocess.Popen(cmd, cwd=ROOT, env=cenv, stdout=subprocess.PIPE,
                                          stderr=subprocess.PIPE, text=True))
        _wait_ready([f"{tmp}/ready{i}" for i in range(a.clients)], procs + [server], deadline, "group clients")
        with open(f"{tmp}/go.tmp", "w") as f:
            f.write(f"{time.time() + 0.5:.6f}")
        os.replace(f"{tmp}/go.tmp", f"{tmp}/go")
        clients = []
        for p in procs:
            out, err = p.communicate(timeout=a.timeout)
            js = [ln for ln in out.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not js:
                raise RuntimeError(f"group client failed rc={p.returncode}: {err[-1500:]}")
            clients.append(json.loads(js[-1]))
        from ..serving import client as sc

        res["server"] = sc.call(endpoint, {"op": "stats"})
        sc.call(endpoint, {"op": "shutdown"})
        server.communicate(timeout=30)
    finally:
        if server.poll() is None:
            server.kill()
    t0 = min(c["t_start"] for c in clients)
    t1 = max(c["t_end"] for c in clients)
    toks = sum(c["tokens"] for c in clients)
    agg = toks / (t1 - t0)
    res.update({
        "per_client_tokens_per_s": [round(c["tokens_per_s"], 1) for c in clients],
        "per_client_step_ms": [round(c["step_ms"], 3) for c in clients],
        "per_client_ttft_ms": [round(1000 * c["ttft_s"], 1) for c in clients],
        "aggregate_tokens_per_s": round(agg, 1),
        # from the first submit to the last token: prefill of all eight included
        "aggregate_tokens_per_s_incl_prefill": round(
            sum(c["tokens"] + c["batch"] for c in clients) / (t1 - min(c["t_submit"] for c in clients)), 1),
        "memory_caps_applied": bool(res["server"].get("peak_mem_gb", 0) > 0 and res["hbm_cap"]),
        "server_peak_mem_gb": round(res["server"].get("peak_mem_gb", 0.0), 2),
    })
    if not a.skip_baselines:
        alone = res["alone"]["tokens_per_s"]
        res.update({"alone_tokens_per_s": round(alone, 1), "density_vs_alone": round(agg / alone, 3)})
    return res


def colocate(a) -> dict:
    if a.share_mode == "batched":
        return colocate_batched(a)
    shares, src = place_shares(a.clients, a.cu_percent, a.memory_gb)
    gpus = {s["shared_gpu"] for s in shares}
    masks = [s["env"]["HSA_CU_MASK"] for s in shares]
    res: dict = {"clients": a.clients, "model": a.model, "batch_per_client": a.batch,
                 "prompt": a.prompt, "new_tokens": a.new, "topology_source": src,
                 "shared_gpus": sorted(gpus), "cu_masks": masks, "mask_style": a.mask_style}
    # (a) one client alone on the whole GPU; (b) one process, combined batch
    if not a.skip_baselines:
        res["alone"] = _run_alone(a, a.batch)
        res["one_process_combined_batch"] = _run_alone(a, a.batch * a.clients)
    tmp = tempfile.mkdtemp(prefix="kgwe-coloc-")
    procs = []
    for i, s in enumerate(shares):
        env = dict(os.environ)
        env.update({k: v for k, v in s["env"].items()})
        # one visible device in this single-GPU harness: the pod's HIP index 0
        env["HIP_VISIBLE_DEVICES"] = env["ROCR_VISIBLE_DEVICES"] = "0"
        if a.mask_style == "strided":  # one CU per XCD-stride instead of a contiguous range
            b, e = (int(x) for x in s["env"]["KGWE_CU_RANGE"].split("-"))
            n = e - b
            env["HSA_CU_MASK"] = "0:" + ",".join(str(i + 8 * j) for j in range(n))
        elif a.mask_style == "none":
            env.pop("HSA_CU_MASK", None)
        if a.hw_queues > 0:
            env["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)
        cmd = _client_cmd(a, a.batch) + ["--ready-file", f"{tmp}/ready{i}", "--go-file", f"{tmp}/go"]
        procs.append(subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    deadline = time.time() + a.timeout
    while not all(os.path.exists(f"{tmp}/ready{i}") for i in range(a.clients)):
        if time.time() > deadline or any(p.poll() not in (None, 0) for p in procs):
            for p in procs:
                p.kill()
            errs = [p.communicate()[1][-800:] for p in procs if p.returncode not in (None, 0)]
            raise RuntimeError(f"co-located clients did not get ready: {errs[:2]}")
        time.sleep(0.05)
    with open(f"{tmp}/go.tmp", "w") as f:
        f.write(f"{time.time() + 0.5:.6f}")
    os.replace(f"{tmp}/go.tmp", f"{tmp}/go")
    clients = []
    for p in procs:
        out, err = p.communicate(timeout=a.timeout)
        js = [ln for ln in out.splitlines() if ln.startswith("{")]
        if p.returncode != 0 or not js:
            raise RuntimeError(f"client failed rc={p.returncode}: {err[-1500:]}")
        clients.append(json.loads(js[-1]))
    t0 = min(c["t_start"] for c in clients)
    t1 = max(c["t_end"] for c in clients)
    toks = sum(c["tokens"] for c in clients)
    agg = toks / (t1 - t0)
    res.update({
        "per_client_tokens_per_s": [round(c["tokens_per_s"], 1) for c in clients],
        "per_client_step_ms": [round(c["step_ms"], 3) for c in clients],
        "start_skew_ms": round(1000 * (max(c["t_start"] for c in clients) - t0), 2),
        "aggregate_tokens_per_s": round(agg, 1),
        "hw_queues_per_client": env.get("GPU_MAX_HW_QUEUES"),
        "memory_caps_applied": all(c["share"].get("applied") for c in clients) if a.memory_gb > 0 else None,
        "peak_mem_gb_per_client": [round(c["peak_mem_gb"], 2) for c in clients],
    })
    if not a.skip_baselines:
        alone, comb = res["alone"]["tokens_per_s"], res["one_process_combined_batch"]["tokens_per_s"]
        res.update({"alone_tokens_per_s": round(alone, 1), "combined_batch_tokens_per_s": round(comb, 1),
                    "density_vs_alone": round(agg / alone, 3),
                    "vs_one_process_combined_batch": round(agg / comb, 3)})
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kgwe bench-infer")
    ap.add_argument("mode", choices=["run", "colocate", "client"])
    ap.add_argument("--model", default="llama3.2-1b")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--cu-percent", type=float, default=12.5, help="per share (12.5 = one XCD)")
    ap.add_argument("--memory-gb", type=float, default=30.0, help="HBM cap per share")
    ap.add_argument("--mask-style", default="ledger", choices=["ledger", "strided", "none"])
    ap.add_argument("--timeout", type=float, default=300.0)
    ap.add_argument("--skip-baselines", action="store_true")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES per client (0: the share env's value)")
    ap.add_argument("--ready-file", default="")
    ap.add_argument("--go-file", default="")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--share-mode", default="processes", choices=["processes", "batched"],
                    help="processes: one process (and one copy of the weights) per client, disjoint CU masks; "
                         "batched: the clients are one share group behind one serving process")
    ap.add_argument("--flush", type=int, default=16, help="batched: decode steps per token hand-out")
    ap.add_argument("--endpoint", default="", help="client: the group server's address")
    ap.add_argument("--vocab", type=int, default=32000, help="client: vocabulary size for the synthetic prompt")
    a = ap.parse_args(argv)
    out = run_client(a) if a.mode == "run" else run_group_client(a) if a.mode == "client" else colocate(a)
    print(json.dumps(out) if a.json else json.dumps(out, indent=1), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
