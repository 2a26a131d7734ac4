"""Print the build id of every benchmarked workload's receiver kernels in a library (codeobj.py).

usage: python tools/kernel_ids.py [lib.so] > kernel_ids.json
tools/gpu_profile.sh writes it beside its PMC passes, so tools/pmc_summary.py stamps each record with the
id of the library the box actually profiled."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import ofdm_pkg  # noqa: E402

ofdm_pkg.load()
from ofdm_amd import abi, codeobj  # noqa: E402


def ids(lib=None) -> dict:
    lib = Path(lib) if lib else abi.library_file()
    return {"library": str(lib.relative_to(ROOT) if lib.is_relative_to(ROOT) else lib),
            "ids": {w: codeobj.workload_build_id(lib, w) for w in codeobj.WORKLOAD_KERNELS}}


if __name__ == "__main__":
    print(json.dumps(ids(sys.argv[1] if len(sys.argv) > 1 else None), indent=1))
