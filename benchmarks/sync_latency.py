"""Host wake-up latency of the ways the miner waits for the GPU (event synchronize,
event query spin, stream synchronize, pinned-copy + event): a ~200 us GPU task, then the
wait; latency = host wall time - GPU time of the task.  python benchmarks/sync_latency.py"""
import statistics
import time

import torch


def main():
    dev = torch.device("cuda")
    a = torch.randn(1536, 1536, device=dev)
    pinned = torch.empty(64, dtype=torch.int64, pin_memory=True)
    src = torch.zeros(64, dtype=torch.int64, device=dev)
    for _ in range(20):
        a @ a
    torch.cuda.synchronize()
    # GPU time of the task
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); a @ a; e1.record(); e1.synchronize()
    gpu_us = e0.elapsed_time(e1) * 1e3

    def task():
        a @ a

    modes = {
        "event.synchronize": lambda e: e.synchronize(),
        "event.query spin": lambda e: [None for _ in iter(lambda: e.query(), True)],
        "stream.synchronize": lambda e: torch.cuda.current_stream().synchronize(),
        "device.synchronize": lambda e: torch.cuda.synchronize(),
    }
    for name, wait in modes.items():
        ts = []
        for _ in range(200):
            task()
            e = torch.cuda.Event()
            e.record()
            t = time.perf_counter()
            wait(e)
            ts.append((time.perf_counter() - t) * 1e6)
        print(f"{name:22s} wait median {statistics.median(ts):8.1f} us  (GPU task {gpu_us:.1f} us)")
    # copy to pinned + event (the miner's readbacks)
    ts = []
    for _ in range(200):
        task()
        pinned.copy_(src, non_blocking=True)
        e = torch.cuda.Event(); e.record()
        t = time.perf_counter()
        e.synchronize()
        ts.append((time.perf_counter() - t) * 1e6)
    print(f"{'d2h copy + event':22s} wait median {statistics.median(ts):8.1f} us")
    # tiny kernel round trip (launch + run + wait)
    x = torch.zeros(1, device=dev)
    for name, wait in modes.items():
        ts = []
        for _ in range(200):
            t = time.perf_counter()
            x.add_(1)
            e = torch.cuda.Event(); e.record()
            wait(e)
            ts.append((time.perf_counter() - t) * 1e6)
        print(f"tiny kernel + {name:22s} round trip median {statistics.median(ts):8.1f} us")


if __name__ == "__main__":
    main()
