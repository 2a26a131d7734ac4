"""oracle/ -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference hot path (``ofdm_oracle.c`` -> ``_lib/liboracle.so``) and the
unmodified reference itself behind an ``#include`` harness (``ref_harness.c`` ->
``_ref/libofdm_ref.so``).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker / the timed CPU baseline.
The product library (``ieee-802.11-ofdm-qpsk-simulator_amd``) never imports it.

Parity of the restatement is pinned against the compiled reference and against
``data/Matlab_Output.txt`` (see tests/test_oracle.py and tests/golden/).
"""
from .orc import Oracle, RefLib, ORACLE_DIR, REF_SO, build_oracle, build_ref  # noqa: F401
