"""Host-to-device ceiling on this box: one pinned 1 GiB buffer copied whole and in 2/8 MiB
chunks (one stream, two streams), and pageable memory; prints GB/s per variant."""
import time
import torch

N = 1 << 30
h = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h.fill_(1)
d = torch.empty(N, dtype=torch.uint8, device="cuda")
s2 = [torch.cuda.Stream(), torch.cuda.Stream()]


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return N / best / 1e9


print("whole pinned", round(timed(lambda: d.copy_(h, non_blocking=True)), 1), "GB/s")
for mb in (2, 8, 64):
    ch = mb << 20

    def chunks():
        for i, o in enumerate(range(0, N, ch)):
            with torch.cuda.stream(s2[i & 1]):
                d[o:o + ch].copy_(h[o:o + ch], non_blocking=True)
    print(f"{mb} MiB chunks, 2 streams", round(timed(chunks), 1), "GB/s")
p = torch.ones(N, dtype=torch.uint8)
print("pageable", round(timed(lambda: d.copy_(p)), 1), "GB/s")
print("D2H pinned", round(timed(lambda: h.copy_(d, non_blocking=True)), 1), "GB/s")
