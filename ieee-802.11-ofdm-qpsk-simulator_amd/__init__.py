"""MI355X-native 802.11a OFDM-QPSK Monte-Carlo engine -- host side.

The per-symbol chain of the reference (src/OFDM.c) runs as fused HIP kernels for gfx950 in
libofdm_mi355x.so behind the C ABI of include/ofdm_mi355x.h; this package binds it with ctypes,
drives sweeps (one process per GPU, counters all-reduced over RCCL) and writes the reference's
data/Output_*.txt file surface.  There is no CPU fallback.
"""
from . import abi  # noqa: F401
from .abi import OfdmError, load_library, make_cfg, make_rx_opts  # noqa: F401
from .engine import Engine, SweepResult  # noqa: F401
from .fileio import (decode_message, read_float_array_file, write_bits_file,  # noqa: F401
                     write_float_array_to_file, write_reference_outputs)

__version__ = "0.1.0"
