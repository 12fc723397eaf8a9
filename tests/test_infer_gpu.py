"""Decode kernels and the bf16 inference harness on MI355X: numerics against
fp32 PyTorch references, hipGraph decode against the full forward, and the
co-located serving run (8 CU-masked clients of one GPU placed by the
scheduler ledger)."""
import json
import os
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("B,hq,hkv,d,smax,lens", [
    (3, 32, 8, 64, 300, [1, 77, 300]),
    (2, 32, 8, 128, 1030, [1030, 513]),
    (2, 8, 8, 64, 200, [64, 65]),
    (1, 16, 2, 128, 4096, [4000]),
    (4, 4, 2, 64, 129, [128, 129, 2, 63]),
])
def test_decode_attention_matches_fp32_reference(B, hq, hkv, d, smax, lens):
    from kgwe.ops import decode as dec

    g = torch.Generator(device="cuda").manual_seed(1)
    q = torch.randn(B, hq, d, device="cuda", generator=g).to(torch.bfloat16)
    kc = torch.randn(B, hkv, smax, d, device="cuda", generator=g).to(torch.bfloat16)
    vc = torch.randn(B, hkv, smax, d, device="cuda", generator=g).to(torch.bfloat16)
    ln = torch.tensor(lens, device="cuda", dtype=torch.int32)
    att = dec.DecodeAttention(B, hq, hkv, d, smax, "cuda")
    got = att(q, kc, vc, ln).float()
    want = dec.decode_attention_reference(q, kc, vc, ln).float()
    err = (got - want).abs().max().item()
    assert err < 2e-2, err


def test_rope_append_matches_reference():
    from kgwe.ops import decode as dec
    from kgwe.ops import reference as ref

    B, hq, hkv, d, smax = 3, 32, 8, 64, 100
    g = torch.Generator(device="cuda").manual_seed(2)
    qkv = torch.randn(B, (hq + 2 * hkv) * d, device="cuda", generator=g).to(torch.bfloat16)
    pos = torch.tensor([0, 17, 99], device="cuda", dtype=torch.int32)
    cos, sin = ref.rope_tables(smax, d, 500000.0, "cuda")
    cos, sin = cos.float().contiguous(), sin.float().contiguous()
    kc = torch.zeros(B, hkv, smax, d, device="cuda", dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    q = dec.rope_append(qkv, pos, cos, sin, kc, vc, hq, hkv, d)
    kr = torch.zeros(B, hkv, smax, d, dtype=torch.bfloat16)
    vr = torch.zeros_like(kr)
    qr = dec.rope_append_reference(qkv.cpu(), pos.cpu(), cos.cpu(), sin.cpu(), kr, vr, hq, hkv, d)
    assert (q.cpu().float() - qr.float()).abs().max().item() < 2e-2
    assert (kc.cpu().float() - kr.float()).abs().max().item() < 2e-2  # only the pos rows written
    assert torch.equal(vc.cpu(), vr)


@pytest.mark.parametrize("B,hq,hkv,d,smax,lens", [
    (3, 32, 8, 64, 300, [1, 77, 300]),     # new token in the first / a middle / the last split
    (2, 16, 4, 128, 1030, [1030, 514]),
    (4, 8, 8, 64, 129, [128, 129, 2, 64]),
])
def test_fused_rope_attention_matches_separate_kernels(B, hq, hkv, d, smax, lens):
    """rope_attend (RoPE + KV append + attention + in-kernel split merge, one
    launch) against rope_append + the attention launch: same appended cache
    rows, same output, and the split tickets reset between calls."""
    from kgwe.ops import decode as dec
    from kgwe.ops import reference as ref

    g = torch.Generator(device="cuda").manual_seed(3)
    qkv = torch.randn(B, (hq + 2 * hkv) * d, device="cuda", generator=g).to(torch.bfloat16)
    kc = torch.randn(B, hkv, smax, d, device="cuda", generator=g).to(torch.bfloat16)
    vc = torch.randn(B, hkv, smax, d, device="cuda", generator=g).to(torch.bfloat16)
    cos, sin = ref.rope_tables(smax, d, 500000.0, "cuda")
    cos, sin = cos.float().contiguous(), sin.float().contiguous()
    ln = torch.tensor(lens, device="cuda", dtype=torch.int32)
    att = dec.DecodeAttention(B, hq, hkv, d, smax, "cuda")
    k1, v1 = kc.clone(), vc.clone()
    q = dec.rope_append(qkv, ln - 1, cos, sin, k1, v1, hq, hkv, d)
    want = att(q, k1, v1, ln).float()
    for _ in range(2):  # twice: the tickets must be back at zero after a call
        k2, v2 = kc.clone(), vc.clone()
        got = att.rope_attend(qkv, cos, sin, k2, v2, ln).float()
        assert torch.equal(k2, k1) and torch.equal(v2, v1)
        err = (got - want).abs().max().item()
        assert err < 1e-2, err
    ref_o = dec.decode_attention_reference(q, k1, v1, ln).float()
    assert (got - ref_o).abs().max().item() < 2e-2


@pytest.mark.parametrize("M,N,K,mode", [
    (1, 384, 2048, 0), (4, 3072, 2048, 1), (8, 520, 2048, 1), (4, 2048, 8192, 0),
    (2, 1024, 2048, 3), (4, 4096, 2048, 3), (4, 20000, 2048, 1), (4, 96, 64, 2),
    # 8 < M <= 32: the matrix-core kernel (one K slice; K split over workgroups; ragged N and M)
    (32, 3072, 2048, 1), (32, 2048, 8192, 0), (12, 520, 2048, 1), (32, 8192, 2048, 3), (17, 1000, 4096, 3),
    (32, 96, 64, 2), (9, 20000, 2048, 1), (32, 4096, 14336, 0),
])
def test_gemv_modes_match_fp32_reference(M, N, K, mode):
    from kgwe.ops import decode as dec

    g = torch.Generator(device="cuda").manual_seed(3)
    x = (torch.randn(M, K, device="cuda", generator=g) * 0.5).bfloat16()
    res = (torch.randn(M, K, device="cuda", generator=g) * 0.5).bfloat16() if mode & dec.GEMV_NORM else None
    rows = 2 * N if mode & dec.GEMV_SWIGLU else N
    w = (torch.randn(rows, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    gw = (1 + 0.1 * torch.randn(K, device="cuda", generator=g)).bfloat16()
    h_out = torch.empty_like(x) if res is not None else None
    y = dec.gemv(x, w, mode, res=res, g=gw if mode & dec.GEMV_NORM else None, h_out=h_out)
    torch.cuda.synchronize()
    yr, hr = dec.gemv_reference(x.cpu(), w.cpu(), mode, res=None if res is None else res.cpu(),
                                g=gw.cpu() if mode & dec.GEMV_NORM else None)
    rel = (y.cpu().float() - yr.float()).norm() / yr.float().norm()
    assert rel < 1e-2, rel.item()
    if h_out is not None:
        assert torch.equal(h_out.cpu(), hr)


@pytest.mark.parametrize("M,N,K", [(4, 50000, 2048), (32, 50000, 2048), (13, 50001, 4096)])
def test_gemv_argmax_matches_torch_argmax(M, N, K):
    from kgwe.ops import decode as dec

    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    w[123] = w[77]  # an exact tie: the first index must win, as in torch.argmax
    gw = torch.ones(K, device="cuda", dtype=torch.bfloat16)
    best = torch.zeros(M, dec.argmax_slots(N, M), dtype=torch.long, device="cuda")
    tok = torch.empty(M, dtype=torch.long, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(2):  # a second step overwrites every partial (and finds the split-K tickets at zero)
        dec.gemv(x, w, dec.GEMV_NORM_ARGMAX, g=gw, y=y, best=best)
        dec.argmax_finish(best, tok)
        torch.cuda.synchronize()
        assert torch.equal(tok, y.argmax(-1)), (tok, y.argmax(-1))


@pytest.mark.parametrize("preset,batch", [("tiny", 2), ("llama3.2-1b", 2), ("tiny", 12), ("llama3.2-1b", 32),
                                          ("tiny", 40)])
def test_graph_decode_logits_match_full_forward(preset, batch):
    """batch <= 8: the vector-ALU projections; 8 < batch <= 32: the matrix-core
    ones (a serving batch); past that the GEMM library.  Six graph replays,
    each checked."""
    from kgwe.models import llama
    from kgwe.models.infer import Generator

    torch.manual_seed(0)
    m = llama.build(preset, device="cuda", dtype=torch.bfloat16)
    m.eval()
    gen = Generator(m, batch=batch, max_seq=96, keep_logits=True)
    assert gen.fused == (batch <= 32)  # past 32 rows: library GEMMs, with the fused RoPE + attention launch
    prompt = torch.randint(0, m.cfg.vocab_size, (batch, 40), device="cuda")
    gen.prefill(prompt)
    gen.capture()
    seq = [prompt]
    for t in range(6):
        seq.append(gen.tok.clone()[:, None])
        gen.step()
        torch.cuda.synchronize()
        with torch.no_grad():
            full = m(torch.cat(seq, 1))[:, -1].float()
        got = gen.logits.float()
        rel = (got - full).norm() / full.norm()
        assert rel < 3e-2, (t, rel.item())


@pytest.mark.timeout(400)
def test_eight_colocated_clients_from_the_ledger():
    cmd = [sys.executable, "-m", "kgwe.bench.infer", "colocate", "--clients", "8", "--model", "llama3.2-1b",
           "--batch", "4", "--prompt", "128", "--new", "129", "--warmup", "4", "--json", "--timeout", "240"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=380)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["topology_source"] == "amd-smi"
    assert len(out["shared_gpus"]) == 1 and len(set(out["cu_masks"])) == 8
    ranges = sorted(tuple(int(x) for x in m.split(":")[1].split("-")) for m in out["cu_masks"])
    assert all(a[1] < b[0] for a, b in zip(ranges, ranges[1:]))  # disjoint CU ranges
    assert all(t > 0 for t in out["per_client_tokens_per_s"])   # every client progressed
    assert out["memory_caps_applied"] is True
    # eight processes stream eight copies of the weights: a little over one lone client's
    # rate on a quiet box (profiles/r02_colocate); the bound only catches serialisation
    assert out["aggregate_tokens_per_s"] >= 0.4 * out["alone_tokens_per_s"]


@pytest.mark.timeout(400)
def test_eight_clients_of_one_share_group_decode_behind_one_server():
    """Same-model clients as ONE share group: one CU range, one HBM cap, one
    copy of the weights; the aggregate must clearly beat one client alone."""
    cmd = [sys.executable, "-m", "kgwe.bench.infer", "colocate", "--share-mode", "batched", "--clients", "8",
           "--cu-percent", "100", "--model", "llama3.2-1b", "--batch", "4", "--prompt", "128", "--new", "129",
           "--warmup", "4", "--json", "--timeout", "240"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=380)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["topology_source"] == "amd-smi"
    assert out["roles"].count("leader") == 1 and out["roles"].count("member") == 7
    assert len(out["shared_gpus"]) == 1 and out["cu_masks"] == ["0:0-255"]
    assert out["server"]["served"] == 8 and out["server"]["tokens_out"] == 8 * 4 * 129
    assert out["memory_caps_applied"] and 0 < out["server_peak_mem_gb"] < 30.0
    assert out["density_vs_alone"] >= 2.0, out


def test_batch_server_graph_replays_match_eager_steps_with_admissions_in_between():
    """Three requests for two slots: the third is prefilled (eager kernels)
    between graph replays, into rows another request just left.  Every token
    must equal the same schedule run without a graph."""
    import threading

    from kgwe.models import llama
    from kgwe.serving import client
    from kgwe.serving.batch_server import BatchServer

    torch.manual_seed(0)
    m = llama.build("llama3.2-1b", device="cuda", dtype=torch.bfloat16)
    m.eval()
    g = torch.Generator().manual_seed(1)
    reqs = [(torch.randint(0, m.cfg.vocab_size, (2, P), generator=g).tolist(), n)
            for P, n in ((64, 21), (32, 40), (48, 30))]

    def serve(graph):
        srv = BatchServer(m, slots=2, rows=2, max_seq=160, flush=8, graph=graph)
        addr = srv.listen("127.0.0.1:0")
        socks = [client.connect(addr) for _ in reqs]
        out = [None] * len(reqs)

        def run(i):
            out[i] = client.generate(reqs[i][0], reqs[i][1], sock=socks[i])["tokens"]

        ths = [threading.Thread(target=run, args=(i,)) for i in range(len(reqs))]
        for t in ths:   # queue all three before the loop starts: one admission order in both runs
            t.start()
        deadline = time.time() + 20
        while srv.pending.qsize() < len(reqs) and time.time() < deadline:
            time.sleep(0.01)
        loop = threading.Thread(target=srv.serve_forever, daemon=True)
        loop.start()
        for t in ths:
            t.join(120)
        srv.stop()
        loop.join(10)
        return out, srv.stats()

    eager, _ = serve(False)
    graphed, st = serve(True)
    assert all(o is not None for o in eager + graphed)
    assert [[len(r) for r in o] for o in graphed] == [[n, n] for _, n in reqs]
    assert graphed == eager
    assert st["served"] == 3


def test_hbm_cap_of_a_share_is_enforced_in_a_workload_that_knows_nothing_of_kgwe(tmp_path):
    """`python -m kgwe.launch -- python workload.py`: the placement's HBM cap
    reaches a plain PyTorch script through the start-up hook; past the cap the
    client gets torch.OutOfMemoryError, below it everything works, and a
    neighbour process on the same GPU is not disturbed."""
    ann = tmp_path / "annotations"
    frac = 4.0 / (torch.cuda.get_device_properties(0).total_memory / 2**30)   # a 4 GiB share
    env_json = json.dumps({"KGWE_SHARING": "CoLocate", "KGWE_GPU_MEMORY_FRACTION": f"{frac:.5f}",
                           "HIP_VISIBLE_DEVICES": "0"})
    ann.write_text(f"kgwe.amd.com/rccl-env={json.dumps(env_json)}\n")
    script = tmp_path / "workload.py"
    script.write_text(
        "import os, sys, torch\n"
        "assert 'kgwe' not in sys.modules\n"
        "a = torch.empty(1 << 30, dtype=torch.uint8, device='cuda')   # 1 GiB: inside the share\n"
        "a.fill_(1)\n"
        "try:\n"
        "    b = torch.empty(6 << 30, dtype=torch.uint8, device='cuda')   # 1 + 6 GiB > 4 GiB\n"
        "    print('NO-CAP')\n"
        "except torch.OutOfMemoryError:\n"
        "    print('OOM-AT-CAP')\n"
        "c = torch.empty(1 << 30, dtype=torch.uint8, device='cuda')   # still serving inside the share\n"
        "torch.cuda.synchronize()\n"
        "print('OK', int(a[:8].sum().item()), os.environ.get('KGWE_GPU_MEMORY_CAP_INSTALLED'))\n")
    env = dict(os.environ, KGWE_ANNOTATIONS_FILE=str(ann))
    env.pop("PYTHONPATH", None)
    r = subprocess.run([sys.executable, "-m", "kgwe.launch", "--", sys.executable, str(script)],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-1500:]
    assert "OOM-AT-CAP" in r.stdout and "NO-CAP" not in r.stdout and "OK 8 1" in r.stdout, r.stdout
    # without a placement the same script is not capped
    env2 = dict(os.environ, KGWE_ANNOTATIONS_FILE=str(tmp_path / "absent"))
    r2 = subprocess.run([sys.executable, "-m", "kgwe.launch", "--", sys.executable, str(script)],
                        cwd=ROOT, env=env2, capture_output=True, text=True, timeout=200)
    assert r2.returncode == 0 and "NO-CAP" in r2.stdout, (r2.stdout, r2.stderr[-800:])
