"""spgemm_amd -- MI355X-native TileSpGEMM (gfx950 HIP kernels behind a C ABI).

Drop-in for the GPU path of for-the-juan/SpGEMM: CSR in, CSR out, with the
reference's tiled-CSR intermediate layout (16x16 tiles, u16 local indices,
MSB-first row bitmasks).  See DESIGN.md and include/tsg.h.
"""
from . import _lib  # noqa: F401
from ._lib import TsgError, build, device_count, header_symbols  # noqa: F401

__all__ = ["TsgError", "build", "device_count", "header_symbols"]
