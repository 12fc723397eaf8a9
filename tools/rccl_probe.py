"""Diagnose single-rank RCCL + FSDP2 on the box (prints timings, dumps stacks if stuck)."""
import faulthandler, os, sys, time
faulthandler.dump_traceback_later(100, exit=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
from kgwe.parallel import dist as kd
t = time.time()
info = kd.init(force_group=True)
print("init", time.time() - t, flush=True)
x = torch.ones(1 << 20, device="cuda")
t = time.time(); dist.all_reduce(x); torch.cuda.synchronize(); print("all_reduce", time.time() - t, x[0].item(), flush=True)
y = torch.empty(2 << 20, device="cuda")
t = time.time(); dist.all_gather_into_tensor(y[: 1 << 20], x); torch.cuda.synchronize(); print("all_gather", time.time() - t, flush=True)
t = time.time(); dist.reduce_scatter_tensor(x[: 1 << 20], x); torch.cuda.synchronize(); print("reduce_scatter", time.time() - t, flush=True)
from kgwe.bench.train import Trainer, TrainConfig
tr = Trainer(TrainConfig(model="tiny", seq_len=256, micro_batch=2), info)
for i in range(3):
    t = time.time(); tr.step(); torch.cuda.synchronize(); print("tiny fsdp step", i, time.time() - t, flush=True)
tr = Trainer(TrainConfig(model="llama3.2-1b", seq_len=1024, micro_batch=1), info)
for i in range(3):
    t = time.time(); tr.step(); torch.cuda.synchronize(); print("1b fsdp step", i, time.time() - t, flush=True)
print("ok", flush=True)
