"""BENCH TOOLING: does work on a second stream run concurrently with the
persistent rx kernel (the overlap an RCCL all-gather relies on at N > 1)?
Times the rx launch, a 1 GiB copy and a spin kernel alone, concurrently and
in sequence.  python tools/overlap_probe.py [spin_cycles]"""
import sys, time, json
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import torch
from pptk_amd.rx import RxContext
from harness.synth import make_batch
dev = torch.device('cuda', 0)
n = 16 * 1024 * 1024
b = make_batch('c1500', n, dev)
ctx = RxContext(0, bytes(range(1, 17)))
recs = torch.empty((n, 64), dtype=torch.uint8, device=dev)
h = torch.empty(n, dtype=torch.int64, device=dev)
src = torch.empty(128 * 1024 * 1024 // 8 * 8, dtype=torch.int64, device=dev)
dst = torch.empty_like(src)
side = torch.cuda.Stream(dev)
def rx():
    ctx.batch_device(b['frames'], n, stride=b['stride'], fixed_len=b['fixed_len'], recs=recs, hash_out=h)
def cp():
    with torch.cuda.stream(side):
        dst.copy_(src)
def timed(f, reps=10):
    for _ in range(3): f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps): f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3
res = {}
res['rx'] = timed(rx)
res['copy_1GB'] = timed(cp)
def both():
    rx(); cp()
res['rx_plus_copy_concurrent'] = timed(both)
def seq():
    rx(); torch.cuda.current_stream().synchronize(); cp(); side.synchronize()
res['sequential'] = timed(seq)
# a latency-only side kernel (spins, no memory traffic): co-scheduled with
# the persistent rx grid the pair takes max(rx, spin), serialised rx + spin
cyc = [int(sys.argv[1])] if len(sys.argv) > 1 else [3_000_000]
def spin():
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc[0])
res['spin'] = timed(spin)
def rx_spin():
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc[0])
    rx()
res['spin_then_rx'] = timed(rx_spin)
def rx_then_spin():
    rx()
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc[0])
res['rx_then_spin'] = timed(rx_then_spin)
print(json.dumps({k: round(v, 3) for k, v in res.items()}))
