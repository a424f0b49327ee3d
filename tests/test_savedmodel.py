"""8f-1: the saved Keras Q-networks reader (prisma_amd/savedmodel.py; utils.py:14-99).

Parity unpinned: the reference ships no saved model and TensorFlow is not installed, so the
bundles here are written by savedmodel.write_tensor_bundle from the published format."""
import os

import numpy as np
import pytest
import torch

from prisma_amd import savedmodel as sm
from prisma_amd.policies import StackedQNet
from prisma_amd.topology import Topology


def test_varint_and_entry_round_trip():
    for x in (0, 1, 127, 128, 300, 2 ** 35 + 7):
        assert sm._varint(sm._enc_varint(x), 0) == (x, len(sm._enc_varint(x)))
    e = sm.parse_entry(sm.encode_entry(1, [11, 32], 0, 4096, 1408, 0xDEADBEEF))
    assert e["dtype"] == 1 and e["shape"] == [11, 32] and e["offset"] == 4096 and e["size"] == 1408
    assert e["crc32c"] == 0xDEADBEEF and e["shard_id"] == 0


def test_table_layout(tmp_path):
    """LevelDB table: entries back in key order, footer magic in the last 8 bytes."""
    p = str(tmp_path / "t.index")
    rows = [(b"b/kernel", b"\x01\x02"), (b"", b"\x08\x01"), (b"a", b"x" * 300)]
    sm.write_table(p, rows)
    raw = open(p, "rb").read()
    assert raw[-8:] == bytes.fromhex("57fb808b247547db")
    assert sm.read_table(p) == sorted(rows)


def test_bundle_round_trip_and_corruption(tmp_path):
    rng = np.random.default_rng(0)
    t = {"layer_with_weights-0/kernel/.ATTRIBUTES/VARIABLE_VALUE": rng.standard_normal((11, 32)).astype(np.float32),
         "layer_with_weights-0/bias/.ATTRIBUTES/VARIABLE_VALUE": rng.standard_normal(32).astype(np.float32),
         "step": np.array(12345, dtype=np.int64),
         "cube": rng.standard_normal((2, 3, 5)).astype(np.float64)}
    prefix = str(tmp_path / "node0" / "variables" / "variables")
    sm.write_tensor_bundle(prefix, t)
    got = sm.read_tensor_bundle(prefix)
    assert set(got) == set(t)
    for k in t:
        assert got[k].dtype == t[k].dtype and got[k].shape == t[k].shape and np.array_equal(got[k], t[k])
    data = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    data[5] ^= 1
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(data))
    with pytest.raises(sm.BundleError, match="CRC"):
        sm.read_tensor_bundle(prefix)
    idx = bytearray(open(prefix + ".index", "rb").read())
    idx[3] ^= 1
    open(prefix + ".index", "wb").write(bytes(idx))
    with pytest.raises(sm.BundleError, match="CRC"):
        sm.read_tensor_bundle(prefix)


@pytest.mark.parametrize("name,kind", [("abilene", "buffer"), ("abilene", "routing"), ("geant", "buffer"),
                                       ("abilene_on_geant", "buffer")])
def test_q_networks_round_trip(tmp_path, name, kind):
    """save_all_models' folder layout (final/node<i>) -> load_model -> the same Q values and
    the same packed in-kernel weights."""
    topo = Topology.example(name)
    net = StackedQNet(topo, kind, seed=5, device="cpu")
    nodes = [int(u) for u in topo.overlay_nodes]
    sm.save_q_networks(net, str(tmp_path / "final"), nodes)
    assert sorted(os.listdir(tmp_path / "final")) == sorted(f"node{i}" for i in nodes)
    k0 = sm.read_tensor_bundle(str(tmp_path / "final" / f"node{nodes[0]}" / "variables" / "variables"))
    assert k0["layer_with_weights-0/kernel/.ATTRIBUTES/VARIABLE_VALUE"].shape == (topo.n_overlay, 32)
    last = 4 if kind == "buffer" else 3
    assert k0[f"layer_with_weights-{last}/kernel/.ATTRIBUTES/VARIABLE_VALUE"].shape == (64, int(topo.degrees[nodes[0]]))
    got = sm.load_q_networks(str(tmp_path / "final"), topo, kind)
    assert sorted(got.loaded_nodes) == sorted(nodes)
    for (n1, p1), (n2, p2) in zip(net.named_parameters(), got.named_parameters()):
        assert n1 == n2 and torch.equal(p1, p2), n1
    rng = np.random.default_rng(1)
    B = 64
    node = torch.from_numpy(rng.choice(nodes, B)).long()
    obs = torch.zeros((B, 1 + topo.max_deg), dtype=torch.int32)
    obs[:, 0] = torch.from_numpy(rng.integers(0, topo.n_overlay, B))
    obs[:, 1:] = torch.from_numpy(rng.integers(0, 16260, (B, topo.max_deg)))
    assert torch.equal(net.q_values(obs, node), got.q_values(obs, node))
    if kind == "buffer":
        assert torch.equal(net.pack(), got.pack())
    one = sm.load_q_networks(str(tmp_path / "final"), topo, kind, node=nodes[1])
    assert one.loaded_nodes == [nodes[1]]


def test_layer_shape_mismatch_raises(tmp_path):
    topo = Topology.example("abilene")
    net = StackedQNet(topo, "routing", seed=1, device="cpu")
    sm.save_q_networks(net, str(tmp_path), [0])
    with pytest.raises(sm.BundleError):
        sm.load_q_networks(str(tmp_path), topo, "buffer")          # 4 Dense layers, buffer has 5
