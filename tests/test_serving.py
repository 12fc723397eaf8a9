"""Shared batch server (kgwe.serving): continuous batching must be invisible
to a client — every request gets exactly the tokens a private Generator
would have produced for its prompt, whenever it joined and whoever else was
decoding (reference capability: MPS clients of one GPU,
src/sharing/mig_controller.go:636-678; parity of outputs unpinned there, the
reference launches nothing)."""
import threading
import time

import pytest
import torch

from kgwe.models import llama
from kgwe.models.infer import Generator
from kgwe.serving import client
from kgwe.serving.batch_server import BatchServer


@pytest.fixture(scope="module")
def model():
    torch.manual_seed(3)
    m = llama.build("tiny")
    m.eval()
    return m


def _private(model, prompt, new):
    g = Generator(model, len(prompt), len(prompt[0]) + new + 1)
    return g.generate(torch.tensor(prompt), new, graph=False).tolist()


def _serve(model, slots, rows, max_seq=96, flush=4):
    srv = BatchServer(model, slots, rows, max_seq, flush=flush, graph=False)
    addr = srv.listen("127.0.0.1:0")
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    return srv, addr, t


def test_each_client_gets_its_private_generators_tokens(model):
    V = model.cfg.vocab_size
    g = torch.Generator().manual_seed(0)
    srv, addr, t = _serve(model, slots=3, rows=2)
    try:
        # five requests for three slots, different prompt lengths and token counts, staggered starts
        reqs = [(torch.randint(0, V, (2, P), generator=g).tolist(), n)
                for P, n in ((16, 9), (24, 17), (8, 5), (16, 1), (32, 12))]
        out = [None] * len(reqs)

        def run(i):
            time.sleep(0.03 * i)
            out[i] = client.generate(reqs[i][0], reqs[i][1], addr)

        ths = [threading.Thread(target=run, args=(i,)) for i in range(len(reqs))]
        [x.start() for x in ths]
        [x.join(60) for x in ths]
        for (prompt, n), res in zip(reqs, out):
            assert res is not None
            assert [len(r) for r in res["tokens"]] == [n, n]
            assert res["tokens"] == _private(model, prompt, n)
        st = client.call(addr, {"op": "stats"})
        assert st["served"] == 5 and st["active"] == 0 and st["tokens_out"] == sum(2 * n for _, n in reqs)
    finally:
        srv.stop()
        t.join(5)


def test_a_burst_of_same_shape_requests_shares_one_prefill_pass(model):
    """Requests that wait together and have one prompt length are admitted in
    ONE prefill pass over consecutive slots; a request of another length gets
    its own.  Everybody still receives its private generator's tokens."""
    V = model.cfg.vocab_size
    g = torch.Generator().manual_seed(1)
    srv = BatchServer(model, 4, 2, 96, flush=4, graph=False)
    addr = srv.listen("127.0.0.1:0")   # accepting, not serving yet: the requests queue up
    reqs = [(torch.randint(0, V, (2, P), generator=g).tolist(), n) for P, n in ((16, 7), (16, 11), (16, 3), (24, 5))]
    out = [None] * len(reqs)
    ths = [threading.Thread(target=lambda i=i: out.__setitem__(i, client.generate(reqs[i][0], reqs[i][1], addr)))
           for i in range(len(reqs))]
    [x.start() for x in ths]
    deadline = time.time() + 10
    while srv.pending.qsize() < len(reqs) and time.time() < deadline:
        time.sleep(0.01)
    assert srv.pending.qsize() == len(reqs)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    try:
        [x.join(60) for x in ths]
        for (prompt, n), res in zip(reqs, out):
            assert res is not None and res["tokens"] == _private(model, prompt, n)
        st = client.call(addr, {"op": "stats"})
        assert st["served"] == 4 and st["prefill_passes"] == 2   # three of length 16 together, one of 24
    finally:
        srv.stop()
        t.join(5)


def test_bad_requests_are_refused_without_disturbing_the_batch(model):
    srv, addr, t = _serve(model, slots=2, rows=1)
    try:
        V = model.cfg.vocab_size
        for bad in ({"op": "generate", "prompt": [[1, 2], [3, 4]], "new": 2},          # two rows, server has one
                    {"op": "generate", "prompt": [[1, 2, 3]], "new": 500},             # past the cache
                    {"op": "generate", "prompt": [[1, V]], "new": 2},                  # token out of range
                    {"op": "generate", "prompt": [[]], "new": 2},
                    {"op": "nonsense"}):
            assert "error" in client.call(addr, bad)
        prompt = [[5, 6, 7, 8]]
        assert client.generate(prompt, 6, addr)["tokens"] == _private(model, prompt, 6)
    finally:
        srv.stop()
        t.join(5)
