"""Weights interop: TF2 tensor-bundle checkpoints (tf_checkpoint.py).

Parity against checkpoints TF itself wrote is unpinned (TF not installed, the reference ships none);
pinned here: CRC-32C known answers (RFC 3720), the format constants, reader/writer round trips,
corruption detection, the Keras layer_with_weights ordering, and a model restored from a checkpoint
reproducing the original model's output on the GPU.
"""
import struct

import numpy as np
import pytest
import torch

from realtime_style_transfer_amd import tf_checkpoint as ck
from realtime_style_transfer_amd.plan import init_weights, network_plan


def test_crc32c_known_answers():
    assert ck.crc32c(b"123456789") == 0xE3069283
    assert ck.crc32c(b"\0" * 32) == 0x8A9136AA                 # RFC 3720 B.4
    assert ck.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert ck.crc32c(bytes(range(32))) == 0x46DD794E
    assert ck.crc32c(b"6789", ck.crc32c(b"12345")) == 0xE3069283
    for c in (0, 1, 0xdeadbeef, 0xffffffff):
        assert ck.unmask_crc(ck.mask_crc(c)) == c


def test_bundle_roundtrip_all_dtypes(tmp_path):
    rng = np.random.default_rng(0)
    t = {"a/kernel/.ATTRIBUTES/VARIABLE_VALUE": rng.standard_normal((3, 3, 5, 7)).astype(np.float32),
         "b": rng.standard_normal(11), "c": np.arange(6, dtype=np.int64).reshape(2, 3),
         "d": np.array(7, dtype=np.int32), "e": rng.standard_normal(4).astype(np.float16),
         "save_counter/.ATTRIBUTES/VARIABLE_VALUE": np.array(3, dtype=np.int64)}
    t.update({f"many/{i:04d}": np.full((i % 5 + 1,), i, np.float32) for i in range(3000)})   # > 1 data block
    prefix = tmp_path / "ckpt-1"
    ck.write_checkpoint(prefix, t, object_graph=b"graph-bytes")
    idx = (tmp_path / "ckpt-1.index").read_bytes()
    lo, hi = struct.unpack('<II', idx[-8:])
    assert (hi << 32 | lo) == ck.TABLE_MAGIC
    r = ck.read_checkpoint(prefix, with_strings=True)
    assert r.pop(ck.OBJECT_GRAPH_KEY).item() == b"graph-bytes"
    assert sorted(r) == sorted(t)
    for k in t:
        assert r[k].dtype == t[k].dtype and r[k].shape == t[k].shape and np.array_equal(r[k], t[k])
    assert ck.list_variables(prefix)[0][0] == "a/kernel/.ATTRIBUTES/VARIABLE_VALUE"


def test_bundle_detects_corruption(tmp_path):
    prefix = tmp_path / "w"
    ck.write_checkpoint(prefix, {"x": np.ones(100, np.float32)})
    data = tmp_path / "w.data-00000-of-00001"
    b = bytearray(data.read_bytes())
    b[17] ^= 1
    data.write_bytes(bytes(b))
    with pytest.raises(ValueError, match="checksum"):
        ck.read_checkpoint(prefix)
    assert ck.read_checkpoint(prefix, verify=False)["x"].shape == (100,)
    (tmp_path / "bad.index").write_bytes(b"\0" * 64)
    with pytest.raises(ValueError, match="magic"):
        ck.read_checkpoint(tmp_path / "bad")


def test_keras_weight_order_and_nested_paths(tmp_path):
    plan = network_plan((32, 64, 17), (32, 64, 3), 8, 8)
    ws = init_weights(plan, seed=3)
    attrs = []
    for l in plan.layers:
        attrs.append(["kernel", "bias"])
        if l.norm == 'bn':
            attrs.append(["gamma", "beta", "moving_mean", "moving_variance"])
    ck.save_keras_weights(tmp_path / "latest_epoch_weights", ws, attrs)
    t = ck.read_checkpoint(tmp_path)                        # directory: follows the 'checkpoint' state file
    got = ck.keras_weights(t)
    assert len(got) == len(ws) and all(np.array_equal(a, b) for a, b in zip(got, ws))
    # the same layers nested one level down (a sub-model of a functional model)
    nested = {f"layer_with_weights-1/{k}": v for k, v in t.items() if k.startswith("layer_with_weights")}
    nested["layer_with_weights-0/kernel/.ATTRIBUTES/VARIABLE_VALUE"] = np.zeros((1, 1, 3, 4), np.float32)
    got2 = ck.keras_weights(nested, "layer_with_weights-1")
    assert all(np.array_equal(a, b) for a, b in zip(got2, ws))
    with pytest.raises(ValueError, match="nontrivial"):
        ck.keras_weights(nested, "layer_with_weights-7")


@pytest.mark.gpu
def test_model_restored_from_checkpoint_reproduces_output(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from realtime_style_transfer_amd.plan import synthetic_style_params
    from realtime_style_transfer_amd.styleTransfer import create_style_transfer_model
    ins, outs, br, bf = (32, 64, 17), (32, 64, 3), 8, 8
    plan = network_plan(ins, outs, br, bf)
    a, P = create_style_transfer_model(ins, outs, br, bf, 1, weights=init_weights(plan, seed=5), max_batch=1)
    b, _ = create_style_transfer_model(ins, outs, br, bf, 1, weights=init_weights(plan, seed=6), max_batch=1)
    a.save_weights(tmp_path / "ckpt")
    b.load_weights(tmp_path / "ckpt")
    x = torch.from_numpy(np.random.default_rng(0).random((1,) + ins, dtype=np.float32)).cuda()
    sp = torch.from_numpy(synthetic_style_params(1, 1, P, plan, seed=1)).cuda()
    ya, yb = a({'content': x, 'style_params': sp}), b({'content': x, 'style_params': sp})
    assert torch.equal(ya, yb)


def _crc32c_py(data: bytes, crc: int = 0) -> int:
    """Bitwise CRC-32C (reflected polynomial 0x82F63B78), independent of librst's slicing-by-8 table code."""
    crc ^= 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def _mask_py(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xa282ead8) & 0xFFFFFFFF


def test_string_tensor_checksums_follow_tensorflow(tmp_path):
    """TF's WriteStringTensor (tensor_bundle.cc) stores [varint len]*[masked crc of the lengths][bytes] and
    checksums each length as the fixed-width little-endian uint32 (uint64 above 4 GiB), not the varint;
    the entry checksum covers those fixed-width lengths, then the 4 stored checksum bytes, then the string
    bytes. Known answer worked out here from that algorithm with an independent CRC; a 300-byte object
    graph makes the varint two bytes long, so varint and uint32 checksums would differ."""
    assert _crc32c_py(b"123456789") == 0xE3069283
    graph = bytes(range(256)) + b"x" * 44                      # 300 bytes: varint 0xAC 0x02
    lens = b"\xac\x02"
    len_crc = _crc32c_py(struct.pack('<I', 300))
    stored = struct.pack('<I', _mask_py(len_crc))
    want_raw = lens + stored + graph
    want_entry_crc = _mask_py(_crc32c_py(graph, _crc32c_py(stored, len_crc)))
    assert _crc32c_py(lens) != len_crc                          # the varint form would be wrong
    prefix = tmp_path / "g"
    ck.write_checkpoint(prefix, {"v": np.ones(3, np.float32)}, object_graph=graph)
    entries = dict(ck._read_table(ck._index_path(str(prefix)), True))
    e = ck.BundleEntry.parse(entries[ck.OBJECT_GRAPH_KEY.encode()])
    data = (tmp_path / "g.data-00000-of-00001").read_bytes()
    assert data[e.offset:e.offset + e.size] == want_raw
    assert e.crc32c == want_entry_crc
    r = ck.read_checkpoint(prefix, with_strings=True)             # verify=True accepts TF's layout
    assert r[ck.OBJECT_GRAPH_KEY].item() == graph
    # a corrupted length checksum is detected
    bad = bytearray(data)
    bad[e.offset + 2] ^= 1
    (tmp_path / "g.data-00000-of-00001").write_bytes(bytes(bad))
    with pytest.raises(ValueError):
        ck.read_checkpoint(prefix, with_strings=True)
