"""can a pageable host->device copy on the default stream wait behind a spin kernel on an
unrelated stream? HIP places streams on GPU_MAX_HW_QUEUES hardware queues (4 on the box) round-robin by creation
order, and a hardware queue runs its packets in order: when the spin stream shares a queue with the copy's path,
the copy waits for the spin. For k = 0..7 extra streams created first, a ~0.5 s spin goes on a fresh stream and the
default stream then copies 64 KB pageable host memory to the device (the tiny-arch cond/text copies of the old
eviction test) and, separately, launches one small kernel; each is timed on the host."""
import time

import torch

assert torch.cuda.is_available()
torch.zeros(1, device="cuda")
keep = []
host = torch.randn(16384)  # 64 KB, pageable
print("GPU_MAX_HW_QUEUES default 4; spin ~0.5 s per row")
for k in range(8):
    torch.cuda.synchronize()
    keep += [torch.cuda.Stream() for _ in range(k)]
    spin = torch.cuda.Stream()
    keep.append(spin)
    with torch.cuda.stream(spin):
        torch.cuda._sleep(int(1.0e9))
    t0 = time.perf_counter()
    d = host.to("cuda")  # pageable: staged copy, synchronous for the host
    t_copy = time.perf_counter() - t0
    t0 = time.perf_counter()
    x = torch.ones(4, device="cuda") + 1
    x.sum().item()
    t_kern = time.perf_counter() - t0
    busy = not spin.query()
    torch.cuda.synchronize()
    print(f"streams created before the spin {len(keep) - 1:3d}: pageable H2D {t_copy * 1e3:8.2f} ms, "
          f"default-stream kernel + D2H {t_kern * 1e3:8.2f} ms, spin still busy after both: {busy}", flush=True)
