"""hunddb_amd — MI355X-native batched block-checksum engine for HundDB's utils/crc.

The product is libhundcrc.so (C ABI in include/hundcrc.h: hand-written gfx950
HIP kernels + host runtime).  This package is its Python face: `hunddb_amd.crc`
mirrors the Go utils/crc surface and exposes the batched GPU entries;
`hunddb_amd.shard` splits a batch by block index across ranks.
"""
from . import crc  # noqa: F401
from .crc import (BLOCK_SIZE, CRC_SIZE, AddCRCsToData, AddCRCToBlockData,  # noqa: F401
                  CheckBlockIntegrity, CRCError, FixLastBlockCRC, GetCRC, HundCRCError,
                  SizeAfterAddingCRCs, SizeWithoutCRCs)

__version__ = "0.1.0"
