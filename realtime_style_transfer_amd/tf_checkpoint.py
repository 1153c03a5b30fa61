"""TF2 checkpoint (tensor bundle) reader / writer — weights interop.

The reference persists weights with ``tf.train.Checkpoint`` / ``Model.save_weights`` (TF format,
``tracing/checkpoint.py:21-37``) and restores them with ``Model.load_weights(path)`` /
``Checkpoint.restore`` (``predict_using_checkpoint.py:84``, ``predict_video_using_checkpoint.py``,
``save_using_checkpoint.py:65-68``). A checkpoint ``<prefix>`` is two files:

* ``<prefix>.index`` — an SSTable (LevelDB table format: prefix-compressed key blocks with restart
  points, an index block, a 48-byte footer ending in the magic 0xdb4775248b80fb57; every block
  followed by a type byte and a masked CRC-32C). Key ``""`` holds a ``BundleHeaderProto``; every other
  key is a variable's checkpoint key with a ``BundleEntryProto`` (dtype, shape, shard, offset, size,
  masked CRC-32C of the bytes).
* ``<prefix>.data-00000-of-0000N`` — the raw little-endian tensor bytes.

Keras functional models name their variables ``layer_with_weights-<i>/<attr>/.ATTRIBUTES/VARIABLE_VALUE``
where ``i`` counts the layers that own weights in model order and ``attr`` is the variable's attribute
(``kernel``, ``bias``, ``gamma``, ``beta``, ``moving_mean``, ``moving_variance``, ``depthwise_kernel``);
nested models add their own ``layer_with_weights-<j>/`` prefix. ``keras_weights`` turns such a
subtree back into the ``get_weights()`` list that ``StyleTransferModel.set_weights`` takes.

Third-party format (TensorFlow 2.9 ``core/util/tensor_bundle``, ``core/lib/io/table``; not vendored in
the reference, TF not installed here): **parity unpinned** against files TF wrote — the reference holds
no checkpoints. The reader is pinned by its own writer (round trip), by CRC-32C known answers, and by
the format constants above.
"""
from __future__ import annotations

import re
import struct
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _lib

TABLE_MAGIC = 0xdb4775248b80fb57
_MASK_DELTA = 0xa282ead8
# tensorflow/core/framework/types.proto DataType -> numpy
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64, 10: np.bool_,
           17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
_DT_STRING = 7
_NP_TO_DT = {np.dtype(v): k for k, v in _DTYPES.items()}
OBJECT_GRAPH_KEY = "_CHECKPOINTABLE_OBJECT_GRAPH"
# Keras get_weights() order of the attributes inside one layer
_ATTR_ORDER = {"kernel": 0, "depthwise_kernel": 0, "bias": 1, "gamma": 2, "beta": 3, "moving_mean": 4,
               "moving_variance": 5}


# ------------------------------------------------------------------------------------------ crc32c
def crc32c(data: bytes, crc: int = 0) -> int:
    return int(_lib.load().rst_crc32c_extend(crc, bytes(data), len(data)))


def mask_crc(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + _MASK_DELTA) & 0xFFFFFFFF


def unmask_crc(m: int) -> int:
    r = (m - _MASK_DELTA) & 0xFFFFFFFF
    return ((r >> 17) | (r << 15)) & 0xFFFFFFFF


# ------------------------------------------------------------------------------------------ varints / protobuf
def _varint(buf: bytes, pos: int) -> Tuple[int, int]:
    r, shift = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        r |= (b & 0x7F) << shift
        if b < 0x80:
            return r, pos
        shift += 7


def _enc_varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _pb_fields(buf: bytes):
    """Yield (field_number, wire_type, value) of a serialized protobuf message."""
    pos = 0
    while pos < len(buf):
        key, pos = _varint(buf, pos)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from('<Q', buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = buf[pos:pos + n]
            pos += n
        elif wt == 5:
            v = struct.unpack_from('<I', buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield fn, wt, v


def _pb_varint(fn: int, v: int) -> bytes:
    return _enc_varint(fn << 3) + _enc_varint(v)


def _pb_bytes(fn: int, b: bytes) -> bytes:
    return _enc_varint((fn << 3) | 2) + _enc_varint(len(b)) + b


def _pb_fixed32(fn: int, v: int) -> bytes:
    return _enc_varint((fn << 3) | 5) + struct.pack('<I', v)


class BundleEntry:
    """tensorflow/core/protobuf/tensor_bundle.proto BundleEntryProto."""

    def __init__(self, dtype=0, shape=(), shard_id=0, offset=0, size=0, crc32c=None):
        self.dtype, self.shape, self.shard_id, self.offset, self.size, self.crc32c = \
            dtype, tuple(shape), shard_id, offset, size, crc32c

    @classmethod
    def parse(cls, buf: bytes) -> "BundleEntry":
        e = cls()
        shape = []
        for fn, wt, v in _pb_fields(buf):
            if fn == 1:
                e.dtype = v
            elif fn == 2:                                   # TensorShapeProto
                for f2, _, v2 in _pb_fields(v):
                    if f2 == 2:                             # Dim
                        size = 0
                        for f3, _, v3 in _pb_fields(v2):
                            if f3 == 1:
                                size = v3 - (1 << 64) if v3 >= (1 << 63) else v3
                        shape.append(size)
            elif fn == 3:
                e.shard_id = v
            elif fn == 4:
                e.offset = v
            elif fn == 5:
                e.size = v
            elif fn == 6:
                e.crc32c = v
            elif fn == 7:
                raise ValueError("partitioned (sliced) variables are not supported")
        e.shape = tuple(shape)
        return e

    def serialize(self) -> bytes:
        shp = b''.join(_pb_bytes(2, _pb_varint(1, d)) for d in self.shape)
        out = _pb_varint(1, self.dtype) + _pb_bytes(2, shp)
        if self.shard_id:
            out += _pb_varint(3, self.shard_id)
        if self.offset:
            out += _pb_varint(4, self.offset)
        out += _pb_varint(5, self.size)
        if self.crc32c is not None:
            out += _pb_fixed32(6, self.crc32c)
        return out


# ------------------------------------------------------------------------------------------ SSTable
def _read_block(buf: bytes, offset: int, size: int, verify: bool) -> List[Tuple[bytes, bytes]]:
    data = buf[offset:offset + size]
    btype = buf[offset + size]
    if btype != 0:
        raise ValueError(f"compressed SSTable block (type {btype}) is not supported")
    if verify:
        stored = struct.unpack_from('<I', buf, offset + size + 1)[0]
        if unmask_crc(stored) != crc32c(data + bytes([btype])):
            raise ValueError(f"SSTable block at {offset}: checksum mismatch")
    nrest = struct.unpack_from('<I', data, len(data) - 4)[0]
    limit = len(data) - 4 - 4 * nrest
    pos, key, out = 0, b'', []
    while pos < limit:
        shared, pos = _varint(data, pos)
        non_shared, pos = _varint(data, pos)
        vlen, pos = _varint(data, pos)
        key = key[:shared] + data[pos:pos + non_shared]
        pos += non_shared
        out.append((key, data[pos:pos + vlen]))
        pos += vlen
    return out


def _read_table(path: Path, verify: bool) -> List[Tuple[bytes, bytes]]:
    buf = Path(path).read_bytes()
    if len(buf) < 48:
        raise ValueError(f"{path}: too short for an SSTable")
    lo, hi = struct.unpack_from('<II', buf, len(buf) - 8)
    if (hi << 32 | lo) != TABLE_MAGIC:
        raise ValueError(f"{path}: not an SSTable (bad magic)")
    pos = len(buf) - 48
    _meta_off, pos = _varint(buf, pos)
    _meta_size, pos = _varint(buf, pos)
    idx_off, pos = _varint(buf, pos)
    idx_size, pos = _varint(buf, pos)
    entries = []
    for _, handle in _read_block(buf, idx_off, idx_size, verify):
        off, p = _varint(handle, 0)
        size, _ = _varint(handle, p)
        entries += _read_block(buf, off, size, verify)
    return entries


class _BlockBuilder:
    def __init__(self, restart_interval=16):
        self.buf, self.restarts, self.counter, self.last, self.ri = bytearray(), [0], 0, b'', restart_interval

    def add(self, key: bytes, value: bytes):
        shared = 0
        if self.counter < self.ri:
            n = min(len(self.last), len(key))
            while shared < n and self.last[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        self.buf += _enc_varint(shared) + _enc_varint(len(key) - shared) + _enc_varint(len(value))
        self.buf += key[shared:] + value
        self.last, self.counter = key, self.counter + 1

    def finish(self) -> bytes:
        return bytes(self.buf) + b''.join(struct.pack('<I', r) for r in self.restarts) + \
            struct.pack('<I', len(self.restarts))

    def empty(self) -> bool:
        return len(self.buf) == 0


def _write_table(path: Path, items: List[Tuple[bytes, bytes]], block_size: int = 262144):
    out = bytearray()

    def emit(block: bytes) -> bytes:
        off = len(out)
        out.extend(block)
        out.append(0)
        out.extend(struct.pack('<I', mask_crc(crc32c(block + b'\0'))))
        return _enc_varint(off) + _enc_varint(len(block))

    index, data = _BlockBuilder(restart_interval=1), _BlockBuilder()
    last_key = b''
    for k, v in items:
        data.add(k, v)
        last_key = k
        if len(data.buf) >= block_size:
            index.add(last_key, emit(data.finish()))
            data = _BlockBuilder()
    if not data.empty():
        index.add(last_key, emit(data.finish()))
    meta = emit(_BlockBuilder().finish())
    idx = emit(index.finish())
    footer = (meta + idx).ljust(40, b'\0') + struct.pack('<II', TABLE_MAGIC & 0xFFFFFFFF, TABLE_MAGIC >> 32)
    out.extend(footer)
    Path(path).write_bytes(bytes(out))


# ------------------------------------------------------------------------------------------ bundle
def _index_path(prefix) -> Path:
    p = str(prefix)
    return Path(p if p.endswith('.index') else p + '.index')


def _resolve_prefix(path) -> str:
    """A checkpoint prefix, or a directory holding TF's ``checkpoint`` state file (latest checkpoint)."""
    p = Path(path)
    if p.is_dir():
        state = p / "checkpoint"
        if not state.exists():
            raise FileNotFoundError(f"{p}: no 'checkpoint' state file")
        m = re.search(r'^model_checkpoint_path:\s*"([^"]+)"', state.read_text(), re.M)
        if not m:
            raise ValueError(f"{state}: no model_checkpoint_path")
        q = Path(m.group(1))
        return str(q if q.is_absolute() else p / q)
    s = str(p)
    return s[:-len('.index')] if s.endswith('.index') else s


def read_checkpoint(path, verify: bool = True, with_strings: bool = False) -> Dict[str, np.ndarray]:
    """All tensors of a TF2 checkpoint: {checkpoint key: array} (tf.train.load_checkpoint + get_tensor)."""
    prefix = _resolve_prefix(path)
    entries = _read_table(_index_path(prefix), verify)
    if not entries or entries[0][0] != b'':
        raise ValueError(f"{prefix}: missing BundleHeaderProto")
    num_shards = 1
    for fn, _, v in _pb_fields(entries[0][1]):
        if fn == 1:
            num_shards = v
        elif fn == 2 and v != 0:
            raise ValueError("big-endian tensor bundles are not supported")
    shards: Dict[int, bytes] = {}
    out: Dict[str, np.ndarray] = {}
    for k, v in entries[1:]:
        e = BundleEntry.parse(v)
        key = k.decode()
        if e.shard_id not in shards:
            shards[e.shard_id] = Path(f"{prefix}.data-{e.shard_id:05d}-of-{num_shards:05d}").read_bytes()
        raw = shards[e.shard_id][e.offset:e.offset + e.size]
        if e.dtype == _DT_STRING:
            # string tensors carry their own checksum layout (tensor_bundle.cc ReadStringTensor)
            vals, crc = _decode_strings(raw, e.shape, verify)
            if verify and e.crc32c is not None and unmask_crc(e.crc32c) != crc:
                raise ValueError(f"{key}: tensor checksum mismatch")
            if with_strings:
                out[key] = vals
            continue
        if verify and e.crc32c is not None and unmask_crc(e.crc32c) != crc32c(raw):
            raise ValueError(f"{key}: tensor checksum mismatch")
        if e.dtype not in _DTYPES:
            raise ValueError(f"{key}: unsupported dtype enum {e.dtype}")
        out[key] = np.frombuffer(raw, dtype=np.dtype(_DTYPES[e.dtype]).newbyteorder('<')).reshape(e.shape).copy()
    return out


def _length_bytes(n: int) -> bytes:
    """A string length as TF checksums it: the in-memory little-endian uint32 (uint64 above 4 GiB),
    not the varint written to the file (tensor_bundle.cc WriteStringTensor, 'backwards compatibility')."""
    return struct.pack('<I', n) if n <= 0xFFFFFFFF else struct.pack('<Q', n)


def _encode_strings(vals) -> Tuple[bytes, int]:
    """On-disk string tensor ``[varint len_0..len_L][masked crc of the lengths][bytes]`` and its entry
    checksum (unmasked): CRC-32C over the fixed-width lengths, then the 4 stored checksum bytes, then the
    string bytes (tensor_bundle.cc WriteStringTensor)."""
    vals = [bytes(v) for v in vals]
    lens = b''.join(_enc_varint(len(v)) for v in vals)
    crc = 0
    for v in vals:
        crc = crc32c(_length_bytes(len(v)), crc)
    stored = struct.pack('<I', mask_crc(crc))
    crc = crc32c(stored, crc)
    for v in vals:
        crc = crc32c(v, crc)
    return lens + stored + b''.join(vals), crc


def _decode_strings(raw: bytes, shape, verify: bool = True) -> Tuple[np.ndarray, int]:
    """Inverse of ``_encode_strings``: (values, entry checksum computed TF's way)."""
    n = int(np.prod(shape)) if shape else 1
    pos, lens, crc = 0, [], 0
    for _ in range(n):
        ln, pos = _varint(raw, pos)
        lens.append(ln)
        crc = crc32c(_length_bytes(ln), crc)
    stored = raw[pos:pos + 4]
    if verify and unmask_crc(struct.unpack('<I', stored)[0]) != crc:
        raise ValueError("string tensor: length checksum mismatch")
    crc = crc32c(stored, crc)
    pos += 4
    vals = []
    for ln in lens:
        vals.append(raw[pos:pos + ln])
        crc = crc32c(raw[pos:pos + ln], crc)
        pos += ln
    return np.array(vals, dtype=object).reshape(shape), crc


def list_variables(path) -> List[Tuple[str, Tuple[int, ...]]]:
    """tf.train.list_variables equivalent (sorted keys, shapes)."""
    return [(k, tuple(v.shape)) for k, v in sorted(read_checkpoint(path).items())]


def write_checkpoint(prefix, tensors: Dict[str, np.ndarray], object_graph: Optional[bytes] = None) -> None:
    """Write a single-shard TF2 tensor bundle (``<prefix>.index`` + ``<prefix>.data-00000-of-00001``)."""
    prefix = str(prefix)
    items = dict(tensors)
    data = bytearray()
    entries = []
    for key in sorted(items):
        a = np.asarray(items[key])          # (np.ascontiguousarray would turn 0-d scalars into shape (1,))
        dt = _NP_TO_DT.get(a.dtype)
        if dt is None:
            raise ValueError(f"{key}: unsupported dtype {a.dtype}")
        raw = a.astype(a.dtype.newbyteorder('<'), copy=False).tobytes(order='C')
        entries.append((key.encode(), BundleEntry(dt, a.shape, 0, len(data), len(raw), mask_crc(crc32c(raw)))))
        data += raw
    if object_graph is not None:
        raw, crc = _encode_strings([object_graph])
        entries.append((OBJECT_GRAPH_KEY.encode(), BundleEntry(_DT_STRING, (), 0, len(data), len(raw),
                                                               mask_crc(crc))))
        data += raw
    entries.sort(key=lambda t: t[0])
    header = _pb_varint(1, 1) + _pb_bytes(3, _pb_varint(1, 1))   # num_shards 1, little-endian, version{producer 1}
    Path(prefix).parent.mkdir(parents=True, exist_ok=True)   # as TF's saver, which creates the checkpoint directory
    Path(f"{prefix}.data-00000-of-00001").write_bytes(bytes(data))
    _write_table(_index_path(prefix), [(b'', header)] + [(k, e.serialize()) for k, e in entries])


# ------------------------------------------------------------------------------------------ Keras mapping
_KEY = re.compile(r'^(?P<path>(?:[^/]+/)*?)layer_with_weights-(?P<i>\d+)/(?P<attr>[A-Za-z_]+)/\.ATTRIBUTES/VARIABLE_VALUE$')


def keras_weights(tensors: Dict[str, np.ndarray], model_path: str = "") -> List[np.ndarray]:
    """The ``get_weights()`` list of the Keras model at ``model_path`` (``""`` = the checkpoint's root;
    e.g. ``"layer_with_weights-1"`` for the second weighted sub-model of a functional model)."""
    pre = model_path.rstrip('/') + '/' if model_path else ''
    found = []
    for k, v in tensors.items():
        m = _KEY.match(k)
        if not m or m.group('path') != pre or m.group('attr') not in _ATTR_ORDER:
            continue
        found.append(((int(m.group('i')), _ATTR_ORDER[m.group('attr')]), v))
    if not found:
        raise ValueError(f"no Keras layer variables under {model_path!r} (assert_nontrivial_match)")
    found.sort(key=lambda t: t[0])
    return [np.asarray(v, dtype=np.float32) for _, v in found]


VAR_SUFFIX = "/.ATTRIBUTES/VARIABLE_VALUE"
SLOT_MARK = "/.OPTIMIZER_SLOT/"


def object_graph_from_keys(keys) -> bytes:
    """A TrackableObjectGraph (trackable_object_graph.proto) for the checkpoint keys of an object-based save.

    Every path component is an ObjectReference (node id, local name) from its parent; a variable node carries
    one SerializedTensor (name "VARIABLE_VALUE", full_name, checkpoint_key). Slot keys
    ``<variable path>/.OPTIMIZER_SLOT/<optimizer path>/<slot>/.ATTRIBUTES/VARIABLE_VALUE`` become slot-variable
    nodes listed by the optimizer node's SlotVariableReferences (original variable node, slot name, slot node).
    Node ids are assigned breadth first, children in first-appearance order, as TF's saver does."""
    children: Dict[tuple, List[str]] = {(): []}
    variables: Dict[tuple, str] = {}
    slots = []                                     # (variable path, optimizer path, slot name, key)

    def add_path(path: tuple):
        for i in range(len(path)):
            parent, name = path[:i], path[i]
            if path[:i + 1] not in children:
                children[path[:i + 1]] = []
                children[parent].append(name)

    for key in keys:
        if key == OBJECT_GRAPH_KEY or not key.endswith(VAR_SUFFIX):
            continue
        body = key[:-len(VAR_SUFFIX)]
        if SLOT_MARK in body:
            var, rest = body.split(SLOT_MARK, 1)
            opt, slot = rest.rsplit('/', 1)
            add_path(tuple(var.split('/')))
            add_path(tuple(opt.split('/')))
            slots.append((tuple(var.split('/')), tuple(opt.split('/')), slot, key))
        else:
            path = tuple(body.split('/'))
            add_path(path)
            variables[path] = key
    ids: Dict[tuple, int] = {(): 0}
    order = [()]
    for path in order:                              # breadth first
        for name in children[path]:
            child = path + (name,)
            ids[child] = len(order)
            order.append(child)
    slot_ids = [len(order) + i for i in range(len(slots))]
    nodes = []
    for path in order:
        msg = b''.join(_pb_bytes(1, _pb_varint(1, ids[path + (n,)]) + _pb_bytes(2, n.encode()))
                       for n in children[path])
        if path in variables:
            msg += _pb_bytes(2, _pb_bytes(1, b"VARIABLE_VALUE") + _pb_bytes(2, "/".join(path).encode()) +
                             _pb_bytes(3, variables[path].encode()))
        for (var, opt, slot, _), sid in zip(slots, slot_ids):
            if opt == path:
                msg += _pb_bytes(3, _pb_varint(1, ids[var]) + _pb_bytes(2, slot.encode()) + _pb_varint(3, sid))
        nodes.append(msg)
    for (var, opt, slot, key) in slots:
        nodes.append(_pb_bytes(2, _pb_bytes(1, b"VARIABLE_VALUE") + _pb_bytes(2, f"{'/'.join(var)}/{slot}".encode()) +
                               _pb_bytes(3, key.encode())))
    return b''.join(_pb_bytes(1, n) for n in nodes)


def parse_object_graph(buf: bytes) -> List[dict]:
    """The nodes of a serialized TrackableObjectGraph: [{'children': [(id, name)], 'keys': [checkpoint_key],
    'slots': [(original id, slot name, slot id)]}] (for tests and inspection)."""
    out = []
    for fn, _, node in _pb_fields(buf):
        if fn != 1:
            continue
        d = {'children': [], 'keys': [], 'slots': []}
        for f2, _, v in _pb_fields(node):
            if f2 == 1:
                ref = dict((f3, v3) for f3, _, v3 in _pb_fields(v))
                d['children'].append((ref.get(1, 0), bytes(ref.get(2, b'')).decode()))
            elif f2 == 2:
                st = dict((f3, v3) for f3, _, v3 in _pb_fields(v))
                d['keys'].append(bytes(st.get(3, b'')).decode())
            elif f2 == 3:
                sr = dict((f3, v3) for f3, _, v3 in _pb_fields(v))
                d['slots'].append((sr.get(1, 0), bytes(sr.get(2, b'')).decode(), sr.get(3, 0)))
        out.append(d)
    return out


def _write_state_file(prefix) -> None:
    """TF's ``checkpoint`` state file (CheckpointState text proto) beside ``prefix``."""
    state = Path(str(prefix)).parent / "checkpoint"
    name = Path(str(prefix)).name
    state.write_text(f'model_checkpoint_path: "{name}"\nall_model_checkpoint_paths: "{name}"\n')


def save_keras_weights(prefix, weights: List[np.ndarray], layer_attrs: List[List[str]]) -> None:
    """Model.save_weights(prefix) (TF format) of a functional model whose weighted layers own the
    attributes ``layer_attrs[i]`` in get_weights() order."""
    tensors = LayerTree(layer_attrs).tensors(weights)
    write_checkpoint(prefix, tensors, object_graph=object_graph_from_keys(tensors))
    _write_state_file(prefix)


# ------------------------------------------------------------------------------------------ Keras layouts
class LayerTree:
    """The weighted layers of a Keras functional model, in model order.

    ``Functional._layer_checkpoint_dependencies`` (Keras 2.9, not vendored) names the i-th layer that owns
    weights ``layer_with_weights-i``, and an object-based checkpoint keys every variable by the first path
    a breadth-first walk from the root reaches it by: ``layer_with_weights-i/<attr>`` for a layer, and
    ``layer_with_weights-i/layer_with_weights-j/<attr>`` for a layer of a sub-model used as a layer (the
    style predictor and the transfer network inside the inference model,
    styleTransferInferenceModel.py:24,37; MobileNetV3Small inside the predictor, stylePrediction.py:33,52).
    An entry is either a list of attribute names (a layer, in its get_weights() order) or a nested LayerTree."""

    def __init__(self, entries):
        self.entries = [e if isinstance(e, LayerTree) else list(e) for e in entries]

    def paths(self, prefix: str = "") -> List[str]:
        """Variable paths (checkpoint keys without the ``/.ATTRIBUTES/VARIABLE_VALUE`` suffix) in the
        model's get_weights() order."""
        out = []
        for i, e in enumerate(self.entries):
            p = f"{prefix}layer_with_weights-{i}/"
            out += e.paths(p) if isinstance(e, LayerTree) else [p + a for a in e]
        return out

    def __len__(self):
        return len(self.paths())

    def tensors(self, weights, prefix: str = "") -> Dict[str, np.ndarray]:
        paths = self.paths(prefix)
        weights = list(weights)
        if len(weights) != len(paths):
            raise ValueError(f"{len(weights)} weights for {len(paths)} layer variables")
        return {p + VAR_SUFFIX: np.asarray(w, np.float32) for p, w in zip(paths, weights)}

    def weights(self, tensors: Dict[str, np.ndarray], prefix: str = "", shapes=None) -> Optional[List[np.ndarray]]:
        """The get_weights() list stored under ``prefix``; None when the checkpoint holds none of these
        variables; ValueError when it holds only some of them or with other shapes (Keras raises on a
        shape mismatch too)."""
        keys = [p + VAR_SUFFIX for p in self.paths(prefix)]
        present = [k in tensors for k in keys]
        if not any(present):
            return None
        if not all(present):
            missing = [k for k, p in zip(keys, present) if not p]
            raise ValueError(f"checkpoint holds {sum(present)} of {len(keys)} variables under {prefix!r}; "
                             f"missing e.g. {missing[:3]}")
        out = [np.asarray(tensors[k], np.float32) for k in keys]
        if shapes is not None:
            got = [tuple(a.shape) for a in out]
            want = [tuple(s) for s in shapes]
            if got != want:
                bad = next(i for i, (g, w) in enumerate(zip(got, want)) if g != w)
                raise ValueError(f"checkpoint variable {keys[bad]} has shape {got[bad]}, the model expects {want[bad]}")
        return out


def layer_tree_from_names(names: List[str]) -> LayerTree:
    """Group ``<layer name>/<attr>`` weight names (get_weights() order) into layers."""
    entries, last = [], None
    for n in names:
        layer, attr = n.rsplit('/', 1)
        if layer != last:
            entries.append([])
            last = layer
        entries[-1].append(attr)
    return LayerTree(entries)


class CheckpointLoadStatus:
    """What ``Model.load_weights`` / ``Checkpoint.restore`` return (TF's CheckpointLoadStatus): which model
    variables were restored, which checkpoint values no model variable took, which model variables the
    checkpoint did not hold."""

    def __init__(self, restored=(), unused=(), missing=()):
        self.restored, self.unused, self.missing = list(restored), list(unused), list(missing)

    def assert_nontrivial_match(self):
        """predict_using_checkpoint.py:85: at least one model variable came from the checkpoint."""
        if not self.restored:
            raise AssertionError("nothing except the root object matched a checkpointed value")
        return self

    def assert_existing_objects_matched(self):
        if self.missing:
            raise AssertionError(f"{len(self.missing)} model variables not in the checkpoint, e.g. {self.missing[:3]}")
        return self

    def assert_consumed(self):
        self.assert_existing_objects_matched()
        if self.unused:
            raise AssertionError(f"unresolved checkpoint values, e.g. {self.unused[:3]}")
        return self

    def expect_partial(self):
        return self

    def run_restore_ops(self, session=None):
        """Eager: the restore already ran."""


class _Part:
    """One sub-model's variables inside a checkpoint: its key prefix, layer tree and weight accessors."""

    def __init__(self, prefix: str, tree: LayerTree, get, set_, shapes):
        self.prefix, self.tree, self.get, self.set, self.shapes = prefix, tree, get, set_, shapes


def parts_tensors(parts) -> Dict[str, np.ndarray]:
    out = {}
    for p in parts:
        out.update(p.tree.tensors(p.get(), p.prefix))
    return out


def restore_parts(parts, tensors: Dict[str, np.ndarray], extra_keys=()) -> CheckpointLoadStatus:
    """Set every part whose variables the checkpoint holds; report the rest. ``extra_keys``: further
    checkpoint keys the caller consumed (optimizer state)."""
    restored, missing, used = [], [], set(extra_keys)
    loaded = []
    for p in parts:
        w = p.tree.weights(tensors, p.prefix, p.shapes)       # raises on a partial / mis-shaped match
        keys = [k + VAR_SUFFIX for k in p.tree.paths(p.prefix)]
        if w is None:
            missing += keys
        else:
            loaded.append((p, w))
            restored += keys
            used.update(keys)
    for p, w in loaded:
        p.set(w)
    unused = [k for k in tensors if k not in used and k != OBJECT_GRAPH_KEY and not k.startswith("save_counter/")]
    return CheckpointLoadStatus(restored, unused, missing)


def save_object(prefix, tensors: Dict[str, np.ndarray], state_file: bool = True) -> str:
    """Write an object-based checkpoint with its TrackableObjectGraph; returns the prefix."""
    write_checkpoint(prefix, tensors, object_graph=object_graph_from_keys(tensors))
    if state_file:
        _write_state_file(prefix)
    return str(prefix)


def latest_checkpoint(checkpoint_dir) -> Optional[str]:
    """tf.train.latest_checkpoint (train_network.py:109): the prefix the directory's state file names."""
    try:
        return _resolve_prefix(Path(checkpoint_dir)) if Path(checkpoint_dir).is_dir() else None
    except (FileNotFoundError, ValueError):
        return None


def load_weights(model, filepath) -> CheckpointLoadStatus:
    """``Model.load_weights(filepath)`` for any mirror model exposing ``_restore_tensors``."""
    return model._restore_tensors(read_checkpoint(filepath))


def save_weights(model, filepath) -> None:
    """``Model.save_weights(filepath)`` (TF format, tracing/checkpoint.py:37)."""
    save_object(filepath, model._checkpoint_tensors())


class Checkpoint:
    """``tf.train.Checkpoint(root)`` / ``tf.train.Checkpoint(name=obj, ...)`` over the mirror models
    (save_using_checkpoint.py:65-66, train_network.py:112-113, tracing/checkpoint.py:21-36). A positional
    root is checkpointed at the top level (Model.save_weights keys); keyword objects under their names.
    ``save`` numbers the prefix with ``save_counter`` (saved as ``save_counter``, int64), ``write`` does not."""

    def __init__(self, root=None, **kwargs):
        self.root = root
        self.named = dict(kwargs)
        self.save_counter = 0

    def _objects(self):
        objs = [("", self.root)] if self.root is not None else []
        return objs + [(f"{k}/", v) for k, v in self.named.items()]

    def _tensors(self) -> Dict[str, np.ndarray]:
        out = {}
        for pre, obj in self._objects():
            out.update({pre + k: v for k, v in obj._checkpoint_tensors().items()})
        out["save_counter" + VAR_SUFFIX] = np.array(self.save_counter, np.int64)
        return out

    def write(self, file_prefix) -> str:
        return save_object(file_prefix, self._tensors(), state_file=False)

    def save(self, file_prefix) -> str:
        self.save_counter += 1
        prefix = f"{file_prefix}-{self.save_counter}"
        save_object(prefix, self._tensors())
        return prefix

    def restore(self, save_path) -> CheckpointLoadStatus:
        if save_path is None:
            return CheckpointLoadStatus()
        tensors = read_checkpoint(save_path)
        restored, missing = [], []
        claimed = set()
        for pre, obj in self._objects():
            sub = {k[len(pre):]: v for k, v in tensors.items() if k.startswith(pre)}
            st = obj._restore_tensors(sub)
            restored += [pre + k for k in st.restored]
            missing += [pre + k for k in st.missing]
            unused_sub = set(st.unused)
            claimed.update(pre + k for k in sub if k not in unused_sub)
        sc = tensors.get("save_counter" + VAR_SUFFIX)
        if sc is not None:
            self.save_counter = int(sc)
            claimed.add("save_counter" + VAR_SUFFIX)
        unused = [k for k in tensors if k not in claimed and k != OBJECT_GRAPH_KEY]
        return CheckpointLoadStatus(restored, unused, missing)

    read = restore


class CheckpointManager:
    """``tf.train.CheckpointManager`` as tracing/checkpoint.py:22-34 uses it: numbered saves
    ``<directory>/<checkpoint_name>-<n>``, the ``checkpoint`` state file, at most ``max_to_keep`` kept.

    As TF's: an existing state file in ``directory`` is read at construction (its checkpoints become the managed list,
    subject to ``max_to_keep``, and ``latest_checkpoint`` names its latest); with ``checkpoint_interval`` (requires
    ``step_counter``: an int, a callable or an object with ``numpy()``/``value``) ``save(check_interval=True)`` writes
    only when the step counter has advanced by at least the interval since the last save — the reference's cadence
    manager (``cadence=10``, train_network.py:70) keeps every 10th epoch, not the last five."""

    def __init__(self, checkpoint: Checkpoint, directory, max_to_keep: Optional[int] = 5,
                 checkpoint_name: str = "ckpt", checkpoint_interval=None, step_counter=None):
        if checkpoint_interval is not None and step_counter is None:
            raise ValueError("`step_counter` should be passed if `checkpoint_interval` is not None.")
        self.checkpoint, self.directory = checkpoint, Path(directory)
        self.max_to_keep, self.checkpoint_name = max_to_keep, checkpoint_name
        self.checkpoint_interval, self._step_counter = checkpoint_interval, step_counter
        self._last_checkpoint_step = None
        self.checkpoints: List[str] = []
        self.directory.mkdir(parents=True, exist_ok=True)
        self._latest = None
        state = self.directory / "checkpoint"
        if state.exists():   # recover the previous run's checkpoints (tf: get_checkpoint_state + _maybe_delete)
            text = state.read_text()
            m = re.search(r'^model_checkpoint_path:\s*"([^"]+)"', text, re.M)
            olds = re.findall(r'^all_model_checkpoint_paths:\s*"([^"]+)"', text, re.M)
            resolve = lambda q: str(Path(q) if Path(q).is_absolute() else self.directory / q)
            self.checkpoints = [resolve(q) for q in olds]
            if m:
                self._latest = resolve(m.group(1))
                if self._latest not in self.checkpoints:
                    self.checkpoints.append(self._latest)

    @property
    def latest_checkpoint(self) -> Optional[str]:
        return self.checkpoints[-1] if self.checkpoints else self._latest

    def _step(self) -> int:
        c = self._step_counter
        if callable(c):
            c = c()
        if hasattr(c, "numpy"):
            c = c.numpy()
        elif hasattr(c, "value") and not isinstance(c, (int, np.integer)):
            c = c.value() if callable(c.value) else c.value
        return int(c)

    def save(self, checkpoint_number=None, check_interval: bool = True) -> Optional[str]:
        # tf.train.CheckpointManager.save: with an interval, a save at the last saved step is always skipped, the
        # interval test applies only when check_interval is set, and every save records its step (a forced save at
        # step 31 moves the next cadence save to >= 31 + interval)
        if self.checkpoint_interval is not None:
            step = self._step()
            if self._last_checkpoint_step is not None:
                if step == self._last_checkpoint_step:
                    return None
                if check_interval and step < self._last_checkpoint_step + self.checkpoint_interval:
                    return None
            self._last_checkpoint_step = step
        n = int(checkpoint_number) if checkpoint_number is not None else self.checkpoint.save_counter + 1
        prefix = self.directory / f"{self.checkpoint_name}-{n}"
        self.checkpoint.save_counter = n
        save_object(prefix, self.checkpoint._tensors(), state_file=False)
        self.checkpoints = [c for c in self.checkpoints if c != str(prefix)] + [str(prefix)]
        while self.max_to_keep is not None and len(self.checkpoints) > self.max_to_keep:
            old = self.checkpoints.pop(0)
            for f in Path(old).parent.glob(Path(old).name + ".*"):
                f.unlink()
        names = [Path(c).name if Path(c).parent == self.directory else c for c in self.checkpoints]
        (self.directory / "checkpoint").write_text(
            f'model_checkpoint_path: "{names[-1]}"\n' + ''.join(f'all_model_checkpoint_paths: "{n}"\n' for n in names))
        return str(prefix)
