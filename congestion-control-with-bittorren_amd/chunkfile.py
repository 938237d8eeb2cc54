"""Chunk-file formats on either side of the hash path.

Parse/emit compatibility only -- no hashing happens here:

    write_chunks(out, digests, first=0)   make_chunks.c:48-53  "%d %s\\n" per chunk
    read_chunk(path)                      chunk.c:93-115       hash column of a chunk file
    find_chunk_idx_from_hash(hex, path)   chunk.c:123-160      index of a hash in a
                                                               chunk / master-chunk file

Formats the reference reads: ``<idx> <40-hex>`` lines (``tmp/*.chunks``,
``tmp/*.haschunks``; the shipped fixtures use CRLF line ends) and the master
chunk file whose first line carries a header in front of chunk 0
(``File: <path> Chunks:0 <hex>``, then ``<idx> <hex>`` lines).
"""
from __future__ import annotations

import os
import sys
from typing import IO, Iterable


def write_chunks(out: str | os.PathLike | IO[str], digests: Iterable[bytes], first: int = 0) -> int:
    """make_chunks.c:48-53: one ``"%d %s\\n"`` line per digest (lowercase
    hex, LF line ends, indices from `first`).  Returns the line count."""
    if isinstance(out, (str, os.PathLike)):
        with open(out, "w", newline="\n") as f:
            return write_chunks(f, digests, first)
    n = 0
    for i, d in enumerate(digests):
        out.write(f"{first + i} {bytes(d).hex()}\n")
        n += 1
    return n


def read_chunk(path: str | os.PathLike) -> list[str]:
    """chunk.c:93-115.  For every line whose first space-separated token
    starts with a digit, the second token with one trailing '\\n' removed
    (a CRLF file keeps its '\\r', as in the reference; the peer compares the
    first 40 characters only).  Other lines, and a digit line without a
    second token (the reference dereferences NULL there), print the
    reference's notice.  Same rules as read_chunk in csrc/chunk_file.c."""
    out = []
    with open(path, "r", newline="") as f:
        for line in f:
            toks = [t for t in line.split(" ") if t != ""]
            if len(toks) >= 2 and toks[0][:1].isdigit():
                tok = toks[1]
                out.append(tok[:-1] if tok.endswith("\n") else tok)
            else:
                sys.stdout.write("Comment line in chunk file\n")
    return out


def _hex_matches(token: str, chunk_hash: str) -> bool:
    # chunk.c:140,149: strcmp(t, hash) == 0 || strstr(t, hash) != NULL
    return token == chunk_hash or chunk_hash in token


def find_chunk_idx_from_hash(chunk_hash: str, hash_chunk_file: str | os.PathLike) -> int:
    """chunk.c:123-160: index of `chunk_hash` in a chunk or master-chunk
    file.  Deviation: on the master file's header line the reference reads
    the index as the first four bytes of the token ``Chunks:0`` (an int
    reinterpretation, chunk.c:138); here it is the number after the colon.
    A hash that is not present raises KeyError (the reference returns an
    uninitialised value)."""
    with open(hash_chunk_file, "r", newline="") as f:
        for line in f:
            toks = [t for t in line.split(" ") if t != ""]
            if not toks:
                continue
            if not toks[0][:1].isdigit():  # header line: File: <path> Chunks:<i> <hex>
                if len(toks) >= 4 and toks[2].startswith("Chunks:"):
                    if _hex_matches(toks[3], chunk_hash):
                        return int(toks[2][len("Chunks:"):])
                continue
            if len(toks) >= 2 and _hex_matches(toks[1], chunk_hash):
                return int(toks[0])
    raise KeyError(f"{chunk_hash} not in {hash_chunk_file}")
