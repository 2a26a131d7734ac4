"""Time the receiver for several symbol-mode configurations (kernel time per launch from the
engine's HIP-event timing), one Tx batch of 5e6 frames, 16 SNR points.

usage: python tools/time_configs.py
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import ofdm_pkg  # noqa: E402

pkg = ofdm_pkg.load()
from ofdm_amd import abi  # noqa: E402

CONFIGS = {
    "ls-real-awgn": dict(est="ls", noise="real", channel="awgn"),
    "ls-complex-awgn": dict(est="ls", noise="complex", channel="awgn"),
    "ls-real-rayleigh": dict(est="ls", noise="real", channel="rayleigh4"),
    "ls-complex-rayleigh": dict(est="ls", noise="complex", channel="rayleigh4"),
    "ideal-real-awgn": dict(est="ideal", noise="real", channel="awgn"),
    "ideal-complex-rayleigh": dict(est="ideal", noise="complex", channel="rayleigh4"),
}


def main():
    frames = 5_000_000
    snr = np.arange(0, 31, 2.0)
    with pkg.Engine(0) as eng:
        counters = eng.new_counters(len(snr))
        tx, bits = eng.tx_buffers(frames)
        for name, kw in CONFIGS.items():
            cfg = pkg.make_cfg(**kw)
            eng.tx_frames(cfg, 0, frames, tx, bits)
            eng.rx_frames(cfg, tx, bits, 0, frames, snr, counters)      # warm
            eng.timing(True)
            eng.timing_reset()
            for _ in range(3):
                eng.rx_frames(cfg, tx, bits, 0, frames, snr, counters)
            eng.timing(False)
            ms, n = eng.timing_query(abi.K_RX)
            units = 2 * frames * len(snr)
            print(f"{name:24s} {ms / n:8.3f} ms/launch  {units / (ms / n * 1e-3):.4g} symbol-SNR/s", flush=True)


if __name__ == "__main__":
    main()
