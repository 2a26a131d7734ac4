"""Where c2's VALU roofline fraction goes below its SNR loop's issue cap: clock, time outside the loop, the loop.

usage: python tools/c2_breakdown.py <bench line json> <stamps txt> <GRBM clock pmc dir> [--out FILE]

  * clock: GRBM_GUI_ACTIVE / 8 XCDs / duration over the receiver dispatches of the same bench command's timed
    steps (all but the warm-up dispatches) -- the bench's fraction is priced at the nominal 2.4 GHz;
  * phases: the OFDM_PACK_STAMPS build's share of wave 0's time (clean spectra and its own Tx in the prologue)
    spent in the SNR loop, and the loop's share of the VALU instructions (isa_mix's loop count per SNR iteration
    x SNR iterations, of the measured SQ_INSTS_VALU per unit);
  * loop: the rest, as the loop's own fraction of the nominal peak at the measured clock, beside its cap.
"""
from __future__ import annotations

import csv
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
NOMINAL_GHZ = 2.4
UNITS_PER_ITERATION = 128      # one SNR iteration of a wave: 64 frames x 2 data symbols


def clock_ghz(pmc_dir: Path, warm: int) -> float:
    rows = [r for f in pmc_dir.glob("**/*counter_collection.csv") for r in csv.DictReader(open(f))
            if "rx_pack_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    rows = rows[warm:]
    cyc = sum(float(r["Counter_Value"]) for r in rows) / 8
    ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
    return cyc / ns


def stamps(path: Path) -> dict:
    """the last cumulative line of wave 0 (the clean-spectrum / own-Tx role)"""
    line = [l for l in path.read_text().splitlines() if l.startswith("pack stamp wave 0")][-1]
    return {k.strip(): float(v) / 100 for k, v in re.findall(r"([a-zA-Z\- ]+) ([0-9.]+)%", line.split(":", 1)[1])}


def main(argv):
    line = json.loads(Path(argv[0]).read_text().strip().splitlines()[-1])
    st = stamps(Path(argv[1]))
    rf = line["roofline"]
    rec = json.loads((ROOT / "profiles" / "pmc_summary.json").read_text())["c2"]
    im = rec["issue_model"]
    ghz = clock_ghz(Path(argv[2]), line["warmup"])
    frac = rf["frac"]
    frac_clk = frac * NOMINAL_GHZ / ghz
    loop_valu_share = im["loop_valu"] / UNITS_PER_ITERATION / rec["valu_instr_per_unit"]
    loop_time = st["SNR loop"]
    loop_frac = frac_clk * loop_valu_share / loop_time
    out = {"bench_line": argv[0], "frac_nominal_clock": frac, "cap": im["cap_frac"], "frac_of_cap": frac / im["cap_frac"],
           "clock_ghz_timed_steps": ghz, "clock_factor": ghz / NOMINAL_GHZ, "frac_at_measured_clock": frac_clk,
           "wave0_time_shares": st, "loop_valu_share": loop_valu_share,
           "loop_frac_at_measured_clock": loop_frac, "loop_frac_of_cap": loop_frac / im["cap_frac"],
           "outside_loop_time": 1 - loop_time, "outside_loop_valu_share": 1 - loop_valu_share}
    text = json.dumps(out, indent=1)
    print(text)
    if "--out" in argv:
        Path(argv[argv.index("--out") + 1]).write_text(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
