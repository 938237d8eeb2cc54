"""MI355X-native SHA-1 chunk-hashing engine for the BitTorrent peer's
hash/verify path (reference: /root/reference sha.c, chunk.c, make_chunks.c,
job.c:217).  The product is the C-ABI library libsha1chunk.so built from
csrc/; this package is its Python view.  Import it with
``importlib.import_module("congestion-control-with-bittorren_amd")``.
"""
from .sha1chunk import *  # noqa: F401,F403
from .sha1chunk import (SHA1, SHA1Context, Sha1ChunkError, binary2hex, device_count,  # noqa: F401
                        get_chunk_hash, hash_batch, hash_device, hash_uniform_device,
                        hex2binary, lib, make_chunks, set_device, shahash,
                        synth_fill_device, verify_batch, verify_hash, VerifyQueue)

__all__ = [
    "SHA1", "SHA1Context", "Sha1ChunkError", "binary2hex", "device_count", "get_chunk_hash",
    "hash_batch", "hash_device", "hash_uniform_device", "hex2binary", "lib", "make_chunks",
    "set_device", "shahash", "synth_fill_device", "verify_batch", "verify_hash", "VerifyQueue",
]
