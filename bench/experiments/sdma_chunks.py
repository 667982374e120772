"""SDMA H2D efficiency vs copy size and stream count (pinned host -> HBM, torch copies):
decides whether a DMA-fed engine could beat the zero-copy feed (55.8 GB/s; SDMA peak 57.3,
profiles/r2/h2d_mix.jsonl)."""
import json
import time

import torch


def main():
    total = 1 << 30
    src = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(total, dtype=torch.uint8, device="cuda")
    for chunk in (256 << 10, 1 << 20, 2 << 20, 4 << 20, 16 << 20):
        for ns in (1, 2, 4):
            streams = [torch.cuda.Stream() for _ in range(ns)]
            n = total // chunk
            for rep in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(n):
                    with torch.cuda.stream(streams[i % ns]):
                        dst[i * chunk:(i + 1) * chunk].copy_(src[i * chunk:(i + 1) * chunk], non_blocking=True)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
            print(json.dumps({"chunk_KB": chunk >> 10, "streams": ns, "GBps": round(total / dt / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
