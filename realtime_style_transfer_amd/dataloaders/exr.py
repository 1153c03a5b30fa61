"""Minimal OpenEXR scanline reader (and writer) — the stand-in for ``pyroexr`` (absent from this image).

The reference reads each Unreal G-buffer channel file with ``pyroexr.load(path)`` and takes
``.channel('R')`` etc. or ``.channels()`` (dataloaders/hdrScreenshots.py:19-25). This module exposes
the same two calls on an :class:`ExrImage`.

Supported (OpenEXR 2 file layout, single-part scanline images): pixel types UINT / HALF / FLOAT,
compression NONE, RLE, ZIPS (1 line per chunk) and ZIP (16 lines per chunk), increasing or
decreasing line order, any data window. Tiled, deep and multi-part files and the lossy / wavelet
codecs (PIZ, PXR24, B44, DWA) raise ``ValueError`` naming the codec. Channels come back as float32
(h, w) arrays (HALF widened exactly, UINT converted).
"""
from __future__ import annotations

import struct
import zlib
from typing import Dict

import numpy as np

MAGIC = 20000630
_COMPRESSION = {0: "NONE", 1: "RLE", 2: "ZIPS", 3: "ZIP", 4: "PIZ", 5: "PXR24", 6: "B44", 7: "B44A", 8: "DWAA",
                9: "DWAB"}
_LINES_PER_CHUNK = {0: 1, 1: 1, 2: 1, 3: 16}
_PIXEL = {0: ('<u4', 4), 1: ('<f2', 2), 2: ('<f4', 4)}


class ExrImage:
    def __init__(self, channels: Dict[str, np.ndarray], header: dict):
        self._channels = channels
        self.header = header

    def channel(self, name: str) -> np.ndarray:
        return self._channels[name]

    def channels(self) -> Dict[str, np.ndarray]:
        return dict(self._channels)

    @property
    def width(self) -> int:
        return next(iter(self._channels.values())).shape[1]

    @property
    def height(self) -> int:
        return next(iter(self._channels.values())).shape[0]


def _cstr(buf: bytes, pos: int):
    end = buf.index(b'\0', pos)
    return buf[pos:end].decode('latin-1'), end + 1


def _parse_header(buf: bytes):
    magic, version = struct.unpack_from('<ii', buf, 0)
    if magic != MAGIC:
        raise ValueError("not an OpenEXR file (bad magic number)")
    if version & 0x200:
        raise ValueError("tiled OpenEXR files are not supported")
    if version & 0x800 or version & 0x1000:
        raise ValueError("deep / multi-part OpenEXR files are not supported")
    pos, attrs = 8, {}
    while buf[pos] != 0:
        name, pos = _cstr(buf, pos)
        typ, pos = _cstr(buf, pos)
        size, = struct.unpack_from('<i', buf, pos)
        pos += 4
        attrs[name] = (typ, buf[pos:pos + size])
        pos += size
    pos += 1
    chans, raw = [], attrs['channels'][1]
    p = 0
    while raw[p] != 0:
        nm, p = _cstr(raw, p)
        ptype, _plin, xs, ys = struct.unpack_from('<iB3xii', raw, p)
        p += 16
        if xs != 1 or ys != 1:
            raise ValueError(f"subsampled channel {nm!r} is not supported")
        chans.append((nm, ptype))
    xmin, ymin, xmax, ymax = struct.unpack('<iiii', attrs['dataWindow'][1])
    comp = attrs['compression'][1][0]
    line_order = attrs['lineOrder'][1][0] if 'lineOrder' in attrs else 0
    return {'channels': chans, 'data_window': (xmin, ymin, xmax, ymax), 'compression': comp,
            'line_order': line_order}, pos


def _unpredict_deinterleave(t: bytes) -> bytes:
    """OpenEXR ZIP/RLE post-processing: undo the byte delta predictor, then the two-half interleave."""
    a = np.frombuffer(t, dtype=np.uint8).astype(np.int64)
    if a.size == 0:
        return b''
    d = a.copy()
    d[1:] -= 128
    u = (np.cumsum(d) & 0xFF).astype(np.uint8)
    half = (u.size + 1) // 2
    out = np.empty_like(u)
    out[0::2] = u[:half]
    out[1::2] = u[half:]
    return out.tobytes()


def _rle_decode(data: bytes, expected: int) -> bytes:
    out = bytearray()
    i = 0
    while i < len(data):
        n = struct.unpack_from('b', data, i)[0]
        i += 1
        if n < 0:
            out += data[i:i - n]
            i += -n
        else:
            out += data[i:i + 1] * (n + 1)
            i += 1
    if len(out) != expected:
        raise ValueError("corrupt RLE chunk")
    return bytes(out)


def load(path) -> ExrImage:
    """pyroexr.load(path) equivalent (scanline files, see module docstring)."""
    buf = open(path, 'rb').read()
    hdr, pos = _parse_header(buf)
    comp = hdr['compression']
    if comp not in _LINES_PER_CHUNK:
        raise ValueError(f"OpenEXR compression {_COMPRESSION.get(comp, comp)} is not supported "
                         f"(supported: NONE, RLE, ZIPS, ZIP)")
    xmin, ymin, xmax, ymax = hdr['data_window']
    w, h = xmax - xmin + 1, ymax - ymin + 1
    lpc = _LINES_PER_CHUNK[comp]
    nchunks = (h + lpc - 1) // lpc
    offsets = struct.unpack_from(f'<{nchunks}Q', buf, pos)
    chans = sorted(hdr['channels'])          # file order is alphabetical by name
    out = {nm: np.empty((h, w), dtype=np.float32) for nm, _ in chans}
    line_bytes = sum(_PIXEL[t][1] for _, t in chans) * w
    for off in offsets:
        y, size = struct.unpack_from('<ii', buf, off)
        data = buf[off + 8: off + 8 + size]
        rows = min(lpc, ymax - y + 1)
        raw_size = rows * line_bytes
        if size < raw_size:
            if comp in (2, 3):
                data = _unpredict_deinterleave(zlib.decompress(data))
            elif comp == 1:
                data = _unpredict_deinterleave(_rle_decode(data, raw_size))
        if len(data) != raw_size:
            raise ValueError(f"corrupt chunk at line {y}")
        p = 0
        for r in range(rows):
            for nm, t in chans:
                dt, sz = _PIXEL[t]
                out[nm][y - ymin + r] = np.frombuffer(data, dtype=dt, count=w, offset=p).astype(np.float32)
                p += sz * w
    return ExrImage(out, hdr)


def save(path, channels: Dict[str, np.ndarray], pixel_type: str = "FLOAT", compression: str = "ZIP") -> None:
    """Write a single-part scanline EXR (NONE / ZIPS / ZIP; HALF or FLOAT) — used to produce test
    inputs and by tools that export G-buffers; ``channels`` maps names to (h, w) arrays."""
    ptype = {"HALF": 1, "FLOAT": 2}[pixel_type]
    comp = {"NONE": 0, "ZIPS": 2, "ZIP": 3}[compression]
    names = sorted(channels)
    h, w = channels[names[0]].shape
    dt, sz = _PIXEL[ptype]

    def attr(name, typ, payload):
        return name.encode() + b'\0' + typ.encode() + b'\0' + struct.pack('<i', len(payload)) + payload

    chl = b''.join(n.encode() + b'\0' + struct.pack('<iB3xii', ptype, 0, 1, 1) for n in names) + b'\0'
    header = struct.pack('<ii', MAGIC, 2)
    header += attr('channels', 'chlist', chl)
    header += attr('compression', 'compression', bytes([comp]))
    header += attr('dataWindow', 'box2i', struct.pack('<iiii', 0, 0, w - 1, h - 1))
    header += attr('displayWindow', 'box2i', struct.pack('<iiii', 0, 0, w - 1, h - 1))
    header += attr('lineOrder', 'lineOrder', bytes([0]))
    header += attr('pixelAspectRatio', 'float', struct.pack('<f', 1.0))
    header += attr('screenWindowCenter', 'v2f', struct.pack('<ff', 0.0, 0.0))
    header += attr('screenWindowWidth', 'float', struct.pack('<f', 1.0))
    header += b'\0'
    lpc = _LINES_PER_CHUNK[comp]
    chunks = []
    for y in range(0, h, lpc):
        rows = min(lpc, h - y)
        raw = b''.join(np.ascontiguousarray(channels[n][y + r], dtype=dt).tobytes()
                       for r in range(rows) for n in names)
        data = raw
        if comp in (2, 3):
            u = np.frombuffer(raw, dtype=np.uint8)
            t = np.concatenate([u[0::2], u[1::2]]).astype(np.int64)   # interleave halves
            d = t.copy()
            d[1:] = (t[1:] - t[:-1] + 128) & 0xFF                     # byte delta predictor
            z = zlib.compress(d.astype(np.uint8).tobytes())
            if len(z) < len(raw):
                data = z
        chunks.append(struct.pack('<ii', y, len(data)) + data)
    table_pos = len(header)
    offs, p = [], table_pos + 8 * len(chunks)
    for c in chunks:
        offs.append(p)
        p += len(c)
    with open(path, 'wb') as f:
        f.write(header + struct.pack(f'<{len(offs)}Q', *offs) + b''.join(chunks))
