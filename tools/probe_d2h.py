"""Probe device->host bandwidth on the GPU box (pageable vs pinned, copy engine vs kernel stores)."""
import time
import torch

n = 49_766_400 // 8
dev = torch.empty(n, dtype=torch.float64, device="cuda").uniform_()
pin = torch.empty(n, dtype=torch.float64, pin_memory=True)
pag = torch.empty(n, dtype=torch.float64)
pag.fill_(0)

def t(fn, k=10):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k

for name, dst in (("pinned", pin), ("pageable", pag)):
    s = t(lambda: dst.copy_(dev, non_blocking=True))
    print(f"D2H {name}: {s*1e3:.3f} ms  {dev.numel()*8/s/1e9:.1f} GB/s", flush=True)
# split over 4 streams
streams = [torch.cuda.Stream() for _ in range(4)]
def split():
    q = n // 4
    for i, st in enumerate(streams):
        with torch.cuda.stream(st):
            pin[i*q:(i+1)*q].copy_(dev[i*q:(i+1)*q], non_blocking=True)
    for st in streams:
        st.synchronize()
s = t(split)
print(f"D2H pinned 4 streams: {s*1e3:.3f} ms  {n*8/s/1e9:.1f} GB/s", flush=True)
s = t(lambda: dev.copy_(pin, non_blocking=True))
print(f"H2D pinned: {s*1e3:.3f} ms  {n*8/s/1e9:.1f} GB/s", flush=True)
