"""Re-stamp profiles/pmc_summary.json records after a change of the build-id definition (not of the code).

usage: python tools/restamp_pmc.py LIB_OF_THE_PROFILED_TREE

Round 3 made the id layout-free (codeobj._layout_free zeroes a descriptor's code-entry offset, which moved
whenever ANY other kernel of the library changed size).  For every record, this script recomputes the OLD
id (plain sha256 over code + descriptor) on a library built from the tree the record was profiled on; only
when that equals the record's id is the record re-stamped with the new id of the same bytes.  The mapping is
written to profiles/r03/pmc/restamp.json.
"""
import hashlib
import importlib.util
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _codeobj():
    spec = importlib.util.spec_from_file_location("codeobj", ROOT / "ieee-802.11-ofdm-qpsk-simulator_amd" / "codeobj.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def old_id(m, lib, wl):
    syms = m.kernel_symbols(lib)
    names = sorted(n for n in syms if any(re.search(re.escape(f), n) for f in m.WORKLOAD_KERNELS[wl]))
    h = hashlib.sha256()
    for n in names:
        h.update(n.encode() + b"\0" + syms[n])
    return h.hexdigest()[:16]


def main(lib):
    m = _codeobj()
    out = ROOT / "profiles" / "pmc_summary.json"
    summary = json.loads(out.read_text())
    mapping = {}
    for wl, rec in summary.items():
        if not isinstance(rec, dict) or wl not in m.WORKLOAD_KERNELS:
            continue
        old, new = old_id(m, lib, wl), m.workload_build_id(lib, wl)
        if rec.get("build_id") != old:
            print(f"{wl}: record {rec.get('build_id')} is not this library's {old}: left as is")
            continue
        mapping[wl] = {"old": old, "new": new}
        rec["build_id"] = new
        rec["build_id_restamped_from"] = old
        im = rec.get("issue_model")
        if im and im.get("build_id") == old:
            im["build_id"] = new
        print(f"{wl}: {old} -> {new}")
    out.write_text(json.dumps(summary, indent=1, sort_keys=True))
    (ROOT / "profiles" / "r03" / "pmc" / "restamp.json").write_text(json.dumps(
        {"library": str(lib), "rule": "old = sha256(code + descriptor); new = codeobj.kernel_build_id "
         "(descriptor code-entry offset zeroed); re-stamped only where old equals the record's id",
         "mapping": mapping}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
