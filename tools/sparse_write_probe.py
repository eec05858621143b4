"""Does the speed of level 1's sparse output pattern depend on the
allocation?  Level 1 writes ~10,100 8-byte records at the start of every
65,536-record tile region (twice: candidate blocks and the band list); this
times that pattern (torch copy kernels, HIP events) on several 8 GB
allocations, against the same bytes written densely.
Usage: python tools/sparse_write_probe.py"""
import json
import torch


def main():
    dev = torch.device("cuda:0")
    tiles, used = 15259, 10096
    src = torch.ones((tiles, used), dtype=torch.int64, device=dev)
    bufs = [torch.empty(tiles * 65536, dtype=torch.int64, device=dev) for _ in range(4)]
    dense = [torch.empty(tiles * used, dtype=torch.int64, device=dev) for _ in range(2)]

    def timed(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    for rnd in range(2):
        for i, b in enumerate(bufs):
            v = b.view(tiles, 65536)[:, :used]
            ms = timed(lambda: v.copy_(src))
            print(json.dumps({"round": rnd, "buf": i, "pattern": "sparse", "ms": round(ms, 4),
                              "gbs": round(tiles * used * 8 / ms / 1e6, 1)}), flush=True)
        for i, d in enumerate(dense):
            v = d.view(tiles, used)
            ms = timed(lambda: v.copy_(src))
            print(json.dumps({"round": rnd, "buf": i, "pattern": "dense", "ms": round(ms, 4),
                              "gbs": round(tiles * used * 8 / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
