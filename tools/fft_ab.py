"""K1 throughput (batched 64-point fft / ifft through ofdm_fft64), for the mapping A/B of DESIGN.md §4.

usage: [OFDM_MI355X_LIB=variants/libofdm_X.so] python tools/fft_ab.py [n_transforms]
Prints transforms/s and the HBM rate (512 B in + 512 B out per transform) from the HIP-event kernel time."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import ofdm_pkg  # noqa: E402


def main(n=1 << 22, reps=20):
    import torch
    pkg = ofdm_pkg.load()
    from ofdm_amd import abi
    eng = pkg.Engine(0)
    x = torch.randn(n, 64, dtype=torch.complex64, device="cuda:0")
    torch.cuda.synchronize()                    # the engine runs on its own stream
    out = {}
    for inv in (False, True):
        for _ in range(3):
            eng.fft64(x, inverse=inv)
        eng.synchronize()
        eng.timing(True)
        eng.timing_reset()
        for _ in range(reps):
            eng.fft64(x, inverse=inv)
        eng.synchronize()
        ms, k = eng.timing_query(abi.K_FFT)
        eng.timing(False)
        t = ms / k / 1e3
        out["ifft" if inv else "fft"] = {"transforms_per_s": n / t, "ms": t * 1e3, "hbm_gbs": n * 1024 / t / 1e9}
    print(json.dumps({"n": n, **out}))
    eng.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22)
