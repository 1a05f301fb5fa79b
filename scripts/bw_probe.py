"""What the HBM delivers to plain streaming kernels on this box (GPU): read-only, copy (1:1) and a 2-read :
1-write stream (torch.add, the tube step's 69 % read / 31 % write mix is between the last two), each over
arrays far larger than the caches, timed with HIP events.  The practical ceiling beside the 8 TB/s peak that
bench.py's roofline fraction is priced against.  usage: python scripts/bw_probe.py [GiB per array]"""
import sys

import torch


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
    n = int(gib * (1 << 30)) // 4
    a = torch.rand(n, device="cuda")
    b = torch.rand(n, device="cuda")
    c = torch.empty_like(a)
    nb = n * 4
    t = timed(lambda: torch.sum(a))
    print(f"read-only (sum)        {nb / t / 1e12:.2f} TB/s")
    t = timed(lambda: c.copy_(a))
    print(f"copy 1 read : 1 write  {2 * nb / t / 1e12:.2f} TB/s")
    t = timed(lambda: torch.add(a, b, out=c))
    print(f"add  2 read : 1 write  {3 * nb / t / 1e12:.2f} TB/s")


if __name__ == "__main__":
    main()
