"""Weights-only import of the reference's saved Keras Q-networks, without TensorFlow.

The reference saves one Keras model per overlay node with ``actor.q_network.save(
f"{folder}/node{i}")`` (prisma/source/utils.py:14-47) and restores them with
``tf.keras.models.load_model`` (utils.py:72-99; forwarder.py:110-114 when ``--load_path`` is set).
A SavedModel keeps its variables as a TensorFlow tensor bundle under
``node{i}/variables/``: ``variables.index`` is a LevelDB-format table (uncompressed blocks of
prefix-compressed keys, restart points, a masked-CRC-32C block trailer, a 48-byte footer with the
table magic) mapping each variable's checkpoint key to a ``BundleEntryProto`` {dtype, shape,
shard_id, offset, size, crc32c}; the key "" holds the ``BundleHeaderProto``; the tensors'
little-endian bytes sit in ``variables.data-<shard>-of-<n>``.

``read_tensor_bundle`` parses that format (every block and tensor CRC checked);
``load_q_networks`` maps each node's Dense layers onto ``policies.StackedQNet`` — Keras keys its
weighted layers ``layer_with_weights-<k>`` in the model's layer order: for DQN_buffer_model
(models.py:258-306) the one-hot branch Dense(32), the buffers branch Dense(32), Dense(64),
Dense(64), Dense(deg); for DQN_routing_model (models.py:360-392) Dense(32), Dense(64), Dense(64),
Dense(deg).  ``write_tensor_bundle`` is the inverse (the tests' fixtures, and a way to hand this
framework's weights back to a TF agent).

Parity unpinned: the reference ships no saved model and TensorFlow is not installed here, so
the reader is checked against bundles this module writes from the published format, not
against a file TensorFlow wrote.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Iterable, List, Tuple

import numpy as np

from .tblog import masked_crc32c

TABLE_MAGIC = 0xDB4775248B80FB57
FOOTER_BYTES = 48
# tensorflow/core/framework/types.proto
DT_NUMPY = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
            10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
DT_STRING = 7
NUMPY_DT = {np.dtype(v): k for k, v in DT_NUMPY.items()}


class BundleError(ValueError):
    pass


# ---------------------------------------------------------------------------
# protobuf wire format (the few messages the bundle uses)
# ---------------------------------------------------------------------------
def _varint(buf: bytes, i: int) -> Tuple[int, int]:
    out, shift = 0, 0
    while True:
        if i >= len(buf):
            raise BundleError("truncated varint")
        b = buf[i]
        i += 1
        out |= (b & 0x7F) << shift
        if not b & 0x80:
            return out, i
        shift += 7


def _enc_varint(x: int) -> bytes:
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _fields(buf: bytes) -> Iterable[Tuple[int, int, object]]:
    """(field number, wire type, value) of a serialized message."""
    i = 0
    while i < len(buf):
        tag, i = _varint(buf, i)
        num, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, i)[0]
            i += 8
        elif wt == 2:
            n, i = _varint(buf, i)
            v = buf[i:i + n]
            i += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, i)[0]
            i += 4
        else:
            raise BundleError(f"unsupported wire type {wt}")
        yield num, wt, v


def parse_entry(buf: bytes) -> dict:
    """BundleEntryProto (tensorflow/core/protobuf/tensor_bundle.proto)."""
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": None, "slices": 0}
    for num, _, v in _fields(buf):
        if num == 1:
            e["dtype"] = v
        elif num == 2:                                   # TensorShapeProto: repeated Dim dim = 2
            for n2, _, d in _fields(v):
                if n2 == 2:
                    size = 0
                    for n3, _, s in _fields(d):
                        if n3 == 1:
                            size = s - (1 << 64) if s >= 1 << 63 else s
                    e["shape"].append(size)
        elif num == 3:
            e["shard_id"] = v
        elif num == 4:
            e["offset"] = v
        elif num == 5:
            e["size"] = v
        elif num == 6:
            e["crc32c"] = v
        elif num == 7:
            e["slices"] += 1
    return e


def _enc_field(num: int, wt: int, payload: bytes) -> bytes:
    return _enc_varint(num << 3 | wt) + payload


def encode_entry(dtype: int, shape: List[int], shard_id: int, offset: int, size: int, crc: int) -> bytes:
    dims = b"".join(_enc_field(2, 2, _enc_varint(len(d)) + d)
                    for d in (_enc_field(1, 0, _enc_varint(s)) for s in shape))
    out = _enc_field(1, 0, _enc_varint(dtype)) + _enc_field(2, 2, _enc_varint(len(dims)) + dims)
    if shard_id:
        out += _enc_field(3, 0, _enc_varint(shard_id))
    if offset:
        out += _enc_field(4, 0, _enc_varint(offset))
    out += _enc_field(5, 0, _enc_varint(size)) + _enc_field(6, 5, struct.pack("<I", crc))
    return out


# ---------------------------------------------------------------------------
# LevelDB table (the .index file)
# ---------------------------------------------------------------------------
def _read_block(data: bytes, offset: int, size: int) -> bytes:
    if offset + size + 5 > len(data):
        raise BundleError("block beyond the end of the index file")
    body = data[offset:offset + size]
    ctype = data[offset + size]
    (crc,) = struct.unpack_from("<I", data, offset + size + 1)
    if masked_crc32c(body + bytes([ctype])) != crc:
        raise BundleError("index block CRC mismatch")
    if ctype != 0:
        raise BundleError(f"compressed index block (type {ctype}) not supported; TF writes them uncompressed")
    return body


def _block_entries(block: bytes) -> List[Tuple[bytes, bytes]]:
    if len(block) < 4:
        raise BundleError("short block")
    (nrest,) = struct.unpack_from("<I", block, len(block) - 4)
    end = len(block) - 4 * (nrest + 1)
    if end < 0:
        raise BundleError("bad restart count")
    out, key, i = [], b"", 0
    while i < end:
        shared, i = _varint(block, i)
        non_shared, i = _varint(block, i)
        vlen, i = _varint(block, i)
        if shared > len(key):
            raise BundleError("bad key prefix")
        key = key[:shared] + block[i:i + non_shared]
        i += non_shared
        out.append((key, block[i:i + vlen]))
        i += vlen
    return out


def read_table(path: str) -> List[Tuple[bytes, bytes]]:
    """Every (key, value) of a LevelDB-format table file, in key order."""
    data = open(path, "rb").read()
    if len(data) < FOOTER_BYTES:
        raise BundleError("index file shorter than its footer")
    foot = data[-FOOTER_BYTES:]
    if struct.unpack_from("<Q", foot, 40)[0] != TABLE_MAGIC:
        raise BundleError("not a LevelDB table (bad magic)")
    i = 0
    _, i = _varint(foot, i)                          # metaindex handle (unused)
    _, i = _varint(foot, i)
    io_, i = _varint(foot, i)
    isz, i = _varint(foot, i)
    out = []
    for _, handle in _block_entries(_read_block(data, io_, isz)):
        off, j = _varint(handle, 0)
        sz, _ = _varint(handle, j)
        out.extend(_block_entries(_read_block(data, off, sz)))
    return out


def _block(entries: List[Tuple[bytes, bytes]]) -> bytes:
    """An uncompressed block, one restart point per entry (no prefix sharing)."""
    body, restarts = bytearray(), []
    for k, v in entries:
        restarts.append(len(body))
        body += _enc_varint(0) + _enc_varint(len(k)) + _enc_varint(len(v)) + k + v
    if not restarts:
        restarts = [0]
    body += b"".join(struct.pack("<I", r) for r in restarts) + struct.pack("<I", len(restarts))
    return bytes(body)


def _with_trailer(body: bytes) -> bytes:
    return body + bytes([0]) + struct.pack("<I", masked_crc32c(body + bytes([0])))


def write_table(path: str, entries: List[Tuple[bytes, bytes]]) -> None:
    entries = sorted(entries)
    data = _block(entries)
    out = bytearray(_with_trailer(data))
    meta_off = len(out)
    meta = _block([])
    out += _with_trailer(meta)
    last = entries[-1][0] if entries else b""
    idx_off = len(out)
    idx = _block([(last, _enc_varint(0) + _enc_varint(len(data)))])
    out += _with_trailer(idx)
    foot = _enc_varint(meta_off) + _enc_varint(len(meta)) + _enc_varint(idx_off) + _enc_varint(len(idx))
    out += foot + bytes(40 - len(foot)) + struct.pack("<Q", TABLE_MAGIC)
    with open(path, "wb") as fh:
        fh.write(out)


# ---------------------------------------------------------------------------
# tensor bundle
# ---------------------------------------------------------------------------
def read_tensor_bundle(prefix: str) -> Dict[str, np.ndarray]:
    """{checkpoint key: array} of the numeric tensors of bundle `prefix` (e.g.
    node0/variables/variables); string tensors (the object graph) are skipped."""
    rows = read_table(prefix + ".index")
    header = dict(rows).get(b"")
    n_shards = 1
    if header is not None:
        for num, _, v in _fields(header):
            if num == 1:
                n_shards = v
    shards: Dict[int, bytes] = {}
    out = {}
    for key, val in rows:
        if key == b"":
            continue
        e = parse_entry(val)
        if e["slices"]:
            raise BundleError(f"{key!r}: partitioned variables are not supported")
        if e["dtype"] == DT_STRING:
            continue
        if e["dtype"] not in DT_NUMPY:
            raise BundleError(f"{key!r}: unsupported dtype {e['dtype']}")
        sid = e["shard_id"]
        if sid not in shards:
            shards[sid] = open(f"{prefix}.data-{sid:05d}-of-{n_shards:05d}", "rb").read()
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        if len(raw) != e["size"]:
            raise BundleError(f"{key!r}: tensor beyond the end of its data file")
        if e["crc32c"] is not None and masked_crc32c(raw) != e["crc32c"]:
            raise BundleError(f"{key!r}: tensor CRC mismatch")
        arr = np.frombuffer(raw, dtype=np.dtype(DT_NUMPY[e["dtype"]]).newbyteorder("<"))
        out[key.decode()] = arr.reshape(e["shape"]).copy()
    return out


def write_tensor_bundle(prefix: str, tensors: Dict[str, np.ndarray]) -> None:
    """One-shard bundle of `tensors` (little-endian, 8-byte aligned as BundleWriter pads)."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    data, rows = bytearray(), []
    for key in sorted(tensors):
        a = np.asarray(tensors[key])
        if a.dtype not in NUMPY_DT:
            raise BundleError(f"{key}: unsupported dtype {a.dtype}")
        raw = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
        data += bytes((-len(data)) % 8)
        rows.append((key.encode(), encode_entry(NUMPY_DT[a.dtype], list(a.shape), 0, len(data), len(raw),
                                                masked_crc32c(raw))))
        data += raw
    header = _enc_field(1, 0, _enc_varint(1))            # num_shards = 1, little endian, version 0
    write_table(prefix + ".index", [(b"", header)] + rows)
    with open(f"{prefix}.data-00000-of-00001", "wb") as fh:
        fh.write(data)


# ---------------------------------------------------------------------------
# Keras Q-networks -> StackedQNet
# ---------------------------------------------------------------------------
def _key(k: int, what: str) -> str:
    return f"layer_with_weights-{k}/{what}/.ATTRIBUTES/VARIABLE_VALUE"


def dense_layers(tensors: Dict[str, np.ndarray]) -> List[Tuple[np.ndarray, np.ndarray]]:
    """(kernel [in, out], bias [out]) of layer_with_weights-0, 1, ... in order."""
    out, k = [], 0
    while _key(k, "kernel") in tensors:
        out.append((tensors[_key(k, "kernel")], tensors[_key(k, "bias")]))
        k += 1
    if not out:
        raise BundleError("no layer_with_weights-<k>/kernel variables: not a saved Keras Dense model")
    return out


def node_index(folder: str) -> int:
    """utils.py:88: int(item.split('_')[-1][4:]) ('node12' -> 12)."""
    return int(folder.split("_")[-1][4:])


def load_q_networks(path: str, topo, kind: str = "buffer", device="cpu", node: int = -1):
    """utils.load_model(path, node_index) for every saved ``node<i>`` folder under `path`, into a
    StackedQNet(topo, kind) (node i = underlay node id, as save_all_models numbers them).  Nodes
    without a folder keep zero weights; a layer whose shape does not fit the node raises."""
    import torch
    from .policies import StackedQNet
    net = StackedQNet(topo, kind, seed=0, device="cpu")
    with torch.no_grad():
        for p in net.parameters():
            p.zero_()
        names = (["W1", "Wb", "W2", "W3", "W4"] if kind == "buffer" else ["W1", "W2", "W3", "W4"])
        loaded = []
        for item in sorted(os.listdir(path)):
            i = node_index(item)
            if node >= 0 and i != node:
                continue
            layers = dense_layers(read_tensor_bundle(os.path.join(path, item, "variables", "variables")))
            if len(layers) != len(names):
                raise BundleError(f"{item}: {len(layers)} Dense layers, the {kind} model has {len(names)}")
            for wn, (K, b) in zip(names, layers):
                W = getattr(net, wn)
                B = getattr(net, "b" + wn[1:])
                if K.ndim != 2 or K.shape[0] > W.shape[1] or K.shape[1] > W.shape[2] or b.shape != (K.shape[1],):
                    raise BundleError(f"{item}: layer {wn} shape {K.shape} does not fit {tuple(W.shape[1:])}")
                W[i, :K.shape[0], :K.shape[1]] = torch.from_numpy(K.astype(np.float32))
                B[i, :K.shape[1]] = torch.from_numpy(b.astype(np.float32))
            loaded.append(i)
    net.loaded_nodes = loaded
    return net.to(device)


def save_q_networks(net, path: str, nodes: Iterable[int]) -> None:
    """The inverse: node<i>/variables/variables.* bundles of StackedQNet `net` in Keras's keys
    (utils.save_all_models' folder layout; variables only, no graph)."""
    names = (["W1", "Wb", "W2", "W3", "W4"] if net.kind == "buffer" else ["W1", "W2", "W3", "W4"])
    deg = net.deg.cpu().numpy()
    for i in nodes:
        t = {}
        for k, wn in enumerate(names):
            W = getattr(net, wn).detach().cpu().numpy()[i]
            b = getattr(net, "b" + wn[1:]).detach().cpu().numpy()[i]
            rows = {"W1": W.shape[0] if wn != "W1" else len(net.topo_overlay_nodes), "Wb": int(deg[i])}.get(wn, W.shape[0])
            cols = int(deg[i]) if wn == "W4" else W.shape[1]
            t[_key(k, "kernel")] = np.ascontiguousarray(W[:rows, :cols])
            t[_key(k, "bias")] = np.ascontiguousarray(b[:cols])
        write_tensor_bundle(os.path.join(path, f"node{i}", "variables", "variables"), t)
