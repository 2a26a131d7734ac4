#!/usr/bin/env python3
"""Frame-sweep packet_idx: GPU against the oracle (TEST INFRASTRUCTURE: loads the oracle as the checker), with every
mismatch checked against Packet_Selection's 0.75 threshold (tests/conftest.off_threshold_pidx_mismatches).  Prints,
per case of tests/test_gpu_frame.py::test_frame_sweep_vs_oracle and tests/test_gpu_message.py, the trials compared,
the mismatches and how many of them the threshold explains, as one JSON object.

usage (GPU box): python tools/pidx_mismatch_report.py [--wide N] > profiles/r06/pidx_mismatches.json
  --wide N: also the reference message over the bench grid (0..30 dB step 2), N trials per point
  --wide8 N: also bench.py's frame8 message (8 data symbols, frame_sync_long_kernel) over the same grid
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import ofdm_pkg  # noqa: E402
from conftest import off_threshold_pidx_mismatches  # noqa: E402
from oracle import Oracle  # noqa: E402


def case(engine, oracle, pkg, abi, msg, snrs, n):
    nd = engine.set_message(msg)
    oracle.set_message(msg)
    w = engine.transmitter("c", "message")
    g, gp = engine.frame_sweep(pkg.make_cfg(payload="message"), snrs, n, want_packet_idx=True)
    o, op = oracle.frame_sweep(oracle.cfg(payload="message"), snrs, 0, n, "c", dump_pidx=True)
    bad = off_threshold_pidx_mismatches(engine, oracle, w, snrs, gp, op, abi.capture_len(nd))
    return {"message_len": len(msg), "data_symbols": nd, "snr_db": list(snrs), "trials": int(gp.size),
            "mismatches": int(np.sum(gp != op)), "unexplained": bad,
            "mismatch_trials": [[int(q), int(t), int(gp[q, t]), int(op[q, t])] for q, t in np.argwhere(gp != op)]}


def main():
    pkg = ofdm_pkg.load()
    from ofdm_amd import abi  # noqa: PLC0415
    oracle = Oracle()
    ref_msg = b"Hey! I am Vivaswan"
    out = []
    with pkg.Engine(0) as e:
        out.append(case(e, oracle, pkg, abi, ref_msg, [6.0, 8.0, 10.0, 14.0], 300))
        out.append(case(e, oracle, pkg, abi, b"IEEE 802.11a on MI355X: a longer message, five symbols!", [8.0, 12.0], 200))
        for msg in (b"Twelve chars", b"x" * 20 + b" three syms", bytes(range(32, 127)) + b"!"):
            out.append(case(e, oracle, pkg, abi, msg, [8.0, 14.0], 160))
        if "--wide" in sys.argv:
            n = int(sys.argv[sys.argv.index("--wide") + 1])
            out.append(case(e, oracle, pkg, abi, ref_msg, [float(x) for x in range(0, 31, 2)], n))
        if "--wide8" in sys.argv:
            from bench import FRAME8_MESSAGE  # noqa: PLC0415
            n = int(sys.argv[sys.argv.index("--wide8") + 1])
            out.append(case(e, oracle, pkg, abi, FRAME8_MESSAGE, [float(x) for x in range(0, 31, 2)], n))
    oracle.set_message(ref_msg)
    print(json.dumps({"generator": "tools/pidx_mismatch_report.py", "cases": out,
                      "total_trials": sum(c["trials"] for c in out),
                      "total_mismatches": sum(c["mismatches"] for c in out),
                      "total_unexplained": sum(len(c["unexplained"]) for c in out)}, indent=1))


if __name__ == "__main__":
    main()
