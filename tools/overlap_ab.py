"""A/B: does the HBM-bound Tx pass (K2) of the next sub-chunk overlap the VALU-bound receiver (K3c) of the
current one when the two go to different HIP streams?  c3 workload (1e7 symbols x 16 SNR points).

usage (GPU box): python tools/overlap_ab.py [--frames 5000000] [--steps 10]
Prints ms per step and symbol-SNR/s for: one chunk in order, N sub-chunks in order, N sub-chunks with the
Tx of sub-chunk k+1 on a second stream (double-buffered Tx batches), and the counters' equality.
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import ofdm_pkg  # noqa: E402

SNR = np.arange(0.0, 31.0, 2.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=5_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--splits", type=int, nargs="*", default=[2, 4, 8])
    args = ap.parse_args()
    import torch
    pkg = ofdm_pkg.load()
    eng = pkg.Engine(0)
    cfg = pkg.make_cfg(est="ls", noise="real", channel="awgn", conv="c", payload="random")
    F = args.frames
    sa = torch.cuda.current_stream(0)
    sb = torch.cuda.Stream(0)

    def run(n_sub, overlap):
        cut = [F * k // n_sub for k in range(n_sub + 1)]
        subs = [(cut[k], cut[k + 1] - cut[k]) for k in range(n_sub)]
        nmax = max(n for _, n in subs)
        bufs = [eng.tx_buffers(nmax) for _ in range(2 if overlap else 1)]
        cnt = eng.new_counters(len(SNR))

        def step():
            cnt.zero_()
            if not overlap:
                for a, n in subs:
                    eng.tx_frames(cfg, a, n, *bufs[0])
                    eng.rx_frames(cfg, *bufs[0], a, n, SNR, cnt)
                return
            tx_done = [torch.cuda.Event() for _ in subs]
            rx_done = [torch.cuda.Event() for _ in subs]
            start = torch.cuda.Event()
            start.record(sa)
            sb.wait_event(start)          # after every receiver of the previous step
            # Tx of sub-chunk 0 on the Rx stream; Tx k+1 on stream B after Rx k-1 freed its buffer
            eng.set_stream(sa.cuda_stream)
            eng.tx_frames(cfg, subs[0][0], subs[0][1], *bufs[0])
            tx_done[0].record(sa)
            for k, (a, n) in enumerate(subs):
                if k + 1 < len(subs):
                    if k >= 1:
                        sb.wait_event(rx_done[k - 1])
                    eng.set_stream(sb.cuda_stream)
                    a1, n1 = subs[k + 1]
                    eng.tx_frames(cfg, a1, n1, *bufs[(k + 1) % 2])
                    tx_done[k + 1].record(sb)
                eng.set_stream(sa.cuda_stream)
                sa.wait_event(tx_done[k])
                eng.rx_frames(cfg, *bufs[k % 2], a, n, SNR, cnt)
                rx_done[k].record(sa)

        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        eng.set_stream(sa.cuda_stream)
        return dt, cnt.cpu().numpy()

    base_t, base_c = run(1, False)
    out = {"one_chunk": {"ms": base_t * 1e3, "rate": 2 * F * len(SNR) / base_t}}
    for n in args.splits:
        for ov in (False, True):
            t, c = run(n, ov)
            out[f"{n}_{'overlap' if ov else 'serial'}"] = {"ms": t * 1e3, "rate": 2 * F * len(SNR) / t,
                                                          "counters_equal": bool(np.array_equal(c, base_c))}
    print(json.dumps(out, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
