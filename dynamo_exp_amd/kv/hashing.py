"""KV block hashing shared by the engine prefix cache, KV events and router.

block hash    = xxh3_64(u32-LE tokens of one full block, seed=1337)
sequence hash = block hash for block 0, else xxh3_64([parent_seq, block] as
                2 x u64-LE, seed=1337)

Identical to the reference (`lib/llm/src/kv_router/indexer.rs:64,87,123`,
`lib/llm/src/tokens.rs:109-243`; test vectors in tests/test_runtime_native.py).
The C++ implementation (`_C_runtime`) is used when built; a pure-Python
fallback over the `xxhash` package keeps CPU CI independent of the build.
"""
from __future__ import annotations

import struct

from .. import _native

KV_HASH_SEED = 1337


def _py():
    import xxhash

    return xxhash


def block_hashes(tokens, block_size: int) -> list[int]:
    rt = _native.runtime()
    if rt is not None:
        return rt.block_hashes(list(tokens), block_size)
    xx = _py()
    n = len(tokens) // block_size
    return [
        xx.xxh3_64_intdigest(struct.pack(f"<{block_size}I", *tokens[i * block_size:(i + 1) * block_size]),
                             seed=KV_HASH_SEED)
        for i in range(n)
    ]


def chain_hashes(block_hashes_: list[int], parent: int | None = None) -> list[int]:
    rt = _native.runtime()
    if rt is not None:
        return rt.chain_hashes(list(block_hashes_), parent)
    xx = _py()
    out = []
    prev = parent
    for b in block_hashes_:
        s = b if prev is None else xx.xxh3_64_intdigest(struct.pack("<2Q", prev, b), seed=KV_HASH_SEED)
        out.append(s)
        prev = s
    return out


def sequence_hashes(tokens, block_size: int, parent: int | None = None) -> list[int]:
    return chain_hashes(block_hashes(tokens, block_size), parent)


def block_and_sequence_hashes(tokens, block_size: int) -> tuple[list[int], list[int]]:
    bh = block_hashes(tokens, block_size)
    return bh, chain_hashes(bh)


def xxh3_64(data: bytes, seed: int = 0) -> int:
    rt = _native.runtime()
    if rt is not None:
        return rt.xxh3_64(data, seed)
    return _py().xxh3_64_intdigest(data, seed=seed)
