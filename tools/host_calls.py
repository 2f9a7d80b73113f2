"""Host cost of the runtime queries on the step's host path (microseconds per
call, median of 200): torch.cuda.mem_get_info (hipMemGetInfo), the allocator
statistics (flattened vs nested), a small pinned-less H2D copy."""
import json
import statistics
import time

import torch


def t(f, n=200):
    xs = []
    for _ in range(n):
        a = time.perf_counter()
        f()
        xs.append((time.perf_counter() - a) * 1e6)
    return round(statistics.median(xs), 1)


def main():
    dev = torch.device("cuda")
    torch.zeros(1, device=dev)
    x = torch.zeros(30, dtype=torch.float32)
    out = {
        "mem_get_info": t(lambda: torch.cuda.mem_get_info()),
        "memory_reserved": t(lambda: torch.cuda.memory_reserved()),
        "memory_stats_as_nested_dict": t(lambda: torch.cuda.memory.memory_stats_as_nested_dict(0)),
        "get_device_properties": t(lambda: torch.cuda.get_device_properties(0).total_memory),
        "h2d_30_floats": t(lambda: x.to(dev, non_blocking=False)),
        "empty_1MB": t(lambda: torch.empty(1 << 18, device=dev)),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
