"""Framing helpers shared by the control plane and the request plane.

* control plane: ``u32-BE length`` + msgpack map per frame;
* request plane: the reference's two-part frame (``u64 header_len, u64
  body_len, u64 xxh3 checksum, header, body`` -- lib/runtime/src/pipeline/
  network/codec/two_part.rs:57-136), encoded/decoded natively by
  ``_C_runtime`` when available.
"""
from __future__ import annotations

import asyncio
import struct

import msgpack

from .. import _native
from ..kv.hashing import xxh3_64

MAX_FRAME = 1 << 30


def pack(obj) -> bytes:
    b = msgpack.packb(obj, use_bin_type=True)
    return struct.pack(">I", len(b)) + b


async def read_frame(reader: asyncio.StreamReader):
    hdr = await reader.readexactly(4)
    (n,) = struct.unpack(">I", hdr)
    if n > MAX_FRAME:
        raise ValueError("frame too large")
    return msgpack.unpackb(await reader.readexactly(n), raw=False, strict_map_key=False)


# ---------------------------------------------------------------- two-part codec
def encode_two_part(header: bytes, body: bytes) -> bytes:
    rt = _native.runtime()
    if rt is not None:
        return rt.encode_two_part(header, body)
    ck = xxh3_64(header + body, 0)
    return struct.pack(">QQQ", len(header), len(body), ck) + header + body


class TwoPartError(Exception):
    pass


async def read_two_part(reader: asyncio.StreamReader, max_size: int = MAX_FRAME) -> tuple[bytes, bytes]:
    pre = await reader.readexactly(24)
    hl, bl, ck = struct.unpack(">QQQ", pre)
    if 24 + hl + bl > max_size:
        raise TwoPartError("message too large")
    data = await reader.readexactly(hl + bl)
    if xxh3_64(data, 0) != ck:
        raise TwoPartError("checksum mismatch")
    return data[:hl], data[hl:]


_PRE = struct.Struct(">QQQ")


async def iter_two_part(reader: asyncio.StreamReader, max_size: int = MAX_FRAME, chunk: int = 1 << 18):
    """Frames from a stream, parsed out of bulk reads: one `read` per burst
    of frames instead of two `readexactly` awaits per frame (the per-token
    frames of hundreds of multiplexed response streams arrive back to back).
    Raises IncompleteReadError at EOF, TwoPartError on a bad frame."""
    buf = bytearray()
    rt = _native.runtime()
    split = getattr(rt, "split_two_part", None) if rt is not None else None
    if split is not None:
        while True:
            try:
                frames, used = split(buf, max_size)
            except (ValueError, RuntimeError) as e:
                raise TwoPartError(str(e)) from None
            if used:
                del buf[:used]
                for f in frames:
                    yield f
            more = await reader.read(chunk)
            if not more:
                raise asyncio.IncompleteReadError(bytes(buf), None)
            buf += more
    pos = 0
    while True:
        while len(buf) - pos >= 24:
            hl, bl, ck = _PRE.unpack_from(buf, pos)
            total = 24 + hl + bl
            if total > max_size:
                raise TwoPartError("message too large")
            if len(buf) - pos < total:
                break
            data = bytes(buf[pos + 24:pos + total])
            if xxh3_64(data, 0) != ck:
                raise TwoPartError("checksum mismatch")
            pos += total
            yield data[:hl], data[hl:]
        if pos:
            del buf[:pos]
            pos = 0
        more = await reader.read(chunk)
        if not more:
            raise asyncio.IncompleteReadError(bytes(buf), None)
        buf += more


def decode_two_part(buf: bytes, max_size: int = 0):
    rt = _native.runtime()
    if rt is not None:
        return rt.decode_two_part(buf, max_size)
    if len(buf) < 24:
        return None
    hl, bl, ck = struct.unpack(">QQQ", buf[:24])
    total = 24 + hl + bl
    if max_size and total > max_size:
        raise TwoPartError("message too large")
    if len(buf) < total:
        return None
    data = buf[24:total]
    if xxh3_64(data, 0) != ck:
        raise TwoPartError("checksum mismatch")
    return data[:hl], data[hl:], total
