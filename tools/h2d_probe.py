"""Host-to-device copy ceiling on this box: pinned host -> HBM rate of one
bench step's input (both views of B frames) split over 1 / 2 / 4 copy streams, at the device
pitch (1280 B rows) and packed (1241 B rows), with the DMA engines (default) or blit kernels
(HSA_ENABLE_SDMA=0, set per run by the parent). Prints one JSON line per configuration.
Usage: python tools/h2d_probe.py [--child STREAMS PITCH]"""
import json
import os
import subprocess
import sys
import time

B, ROWS, COLS = 256, 376, 1241


def child(nstreams, pitch, reps=8):
    import torch
    dev = torch.device("cuda", 0)
    nbytes = 2 * B * ROWS * pitch
    host = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    host.fill_(7)
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(nstreams)]
    chunk = (nbytes + nstreams - 1) // nstreams

    def once():
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                dst[i * chunk:(i + 1) * chunk].copy_(host[i * chunk:(i + 1) * chunk],
                                                    non_blocking=True)
        torch.cuda.synchronize()
    once()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    dt = (time.perf_counter() - t0) / reps
    print(json.dumps({"streams": nstreams, "row_bytes": pitch, "sdma": os.environ.get("HSA_ENABLE_SDMA", "1"),
                      "bytes_per_step": nbytes, "ms_per_step": round(1e3 * dt, 3),
                      "GBps": round(nbytes / dt / 1e9, 2),
                      "stereo_frames_per_s_at_255": round(255 / dt, 1)}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(int(sys.argv[2]), int(sys.argv[3]))
        return
    for sdma in ("1", "0"):
        for pitch in (1280, 1241):
            for ns in (1, 2, 4):
                env = dict(os.environ, HSA_ENABLE_SDMA=sdma)
                p = subprocess.run(["timeout", "-k", "10", "120", sys.executable, __file__,
                                    "--child", str(ns), str(pitch)], env=env, capture_output=True,
                                   text=True)
                if p.returncode != 0:
                    print(json.dumps({"streams": ns, "row_bytes": pitch, "sdma": sdma,
                                      "error": p.stderr[-300:]}), flush=True)
                    sys.exit(1)
                print(p.stdout.strip(), flush=True)


if __name__ == "__main__":
    main()
