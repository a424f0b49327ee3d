"""TensorBoard logging without TensorFlow (prisma_amd/tblog.py; tb_logger.py:15-164).

Framing is pinned by the CRC-32C check value (RFC 3720 B.4: crc32c("123456789") =
0xE3069283) and a byte-level round trip; the tag set by the literal tag lists of
tb_logger.py:96-164; the statistics by an independent recount from the oracle's
decision records of the same notification stream (forwarder.py:197-431 bookkeeping).
"""
import collections
import os

import numpy as np
import pytest

from prisma_amd import tblog
from prisma_amd.config import engine_params
from prisma_amd.topology import Topology, sp_next_hop_table

SESSION_TAGS = [  # tb_logger.py:96-132, in write order
    "total_e2e_delay_over_iterations", "total_e2e_delay_over_time",
    "total_rewards_with_loss_over_iterations", "total_rewards_with_loss_over_time",
    "loss_ratio_over_time", "loss_ratio_over_iterations",
    "total_hops_over_iterations", "total_hops_over_time",
    "avg_hops_over_iterations", "avg_hops_over_time",
    "ma_avg_hops_over_iterations", "ma_avg_hops_over_time",
    "nb_buffered_pkts_over_time", "nb_buffered_pkts_over_iterations",
    "signalling ratio",
    "avg_cost_over_iterations", "avg_cost_over_time",
    "avg_delay_over_iterations", "avg_delay_over_time",
    "ma_delays_over_iterations", "ma_delays_over_time",
    "sim_second_per_real_seconds"]
TEST_TAGS = [  # tb_logger.py:152-164
    "test_global_injected_pkts", "test_overlay_injected_pkts", "test_global_lost_pkts", "test_overlay_lost_pkts",
    "test_global_arrived_pkts", "test_overlay_arrived_pkts", "test_global_e2e_delay", "test_overlay_e2e_delay",
    "test_global_loss_rate", "test_overlay_loss_rate", "test_global_cost", "test_overlay_cost"]


def test_crc32c_check_value_and_masking():
    assert tblog.crc32c(b"") == 0
    assert tblog.crc32c(b"123456789") == 0xE3069283
    assert tblog.crc32c(bytes(32)) == 0x8A9136AA                 # RFC 3720 B.4: 32 bytes of zeros
    c = 0xE3069283
    assert tblog.masked_crc32c(b"123456789") == ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def test_tfrecord_round_trip_and_corruption(tmp_path):
    p = tmp_path / "r.tfrecord"
    payloads = [b"", b"abc", bytes(range(256)) * 3]
    p.write_bytes(b"".join(tblog.tfrecord(x) for x in payloads))
    assert tblog.read_tfrecords(str(p)) == payloads
    b = bytearray(p.read_bytes())
    b[20] ^= 1
    p.write_bytes(bytes(b))
    with pytest.raises(ValueError):
        tblog.read_tfrecords(str(p))


def test_event_writer_scalars(tmp_path):
    w = tblog.EventFileWriter(str(tmp_path / "run"))
    w.scalar("a", 1.5, 3)
    w.scalar("b", -1, 2 ** 40)
    w.close()
    assert os.path.basename(w.path).startswith("events.out.tfevents.") and w.path.endswith(".v2")
    ev = tblog.read_events(w.path)
    assert ev[0]["file_version"] == "brain.Event:2" and not ev[0]["values"]
    assert [(e["step"], e["values"]) for e in ev[1:]] == [(3, [("a", 1.5, "scalars")]),
                                                          (2 ** 40, [("b", -1.0, "scalars")])]


def test_custom_plots_layout():
    s = tblog.Summary.FromString(tblog.custom_plots())
    (v,) = s.value
    assert v.tag == "custom_scalars__config__" and v.metadata.plugin_data.plugin_name == "custom_scalars"
    lay = tblog.Layout.FromString(v.tensor.string_val[0])
    assert [c.title for c in lay.category] == ["Main evaluation metrics", "Training metrics"]
    assert [ch.multiline.tag[0] for c in lay.category for ch in c.chart] == [
        "avg_delay_over_time", "avg_cost_over_time", "loss_ratio_over_time",
        "MSE_loss_over_time", "exploaration_value_over_time", "replay_buffer_length_over_time"]


def test_hparams_record(tmp_path):
    """main.py:79-85: the session parameters (argument_parser.py defaults, G stringified) as the
    hparams plugin's session-start summary in the logs folder, written once at step 0."""
    from prisma_amd.config import parse_arguments
    params = parse_arguments(["--load_factor", "1.5", "--pingAsObs", "0"])
    s = tblog.Summary.FromString(tblog.hparams_summary(params, start_time_secs=12.5))
    (v,) = s.value
    assert v.tag == "_hparams_/session_start_info" and v.metadata.plugin_data.plugin_name == "hparams"
    pd = tblog.HParamsPluginData.FromString(v.metadata.plugin_data.content)
    assert pd.version == 0 and pd.session_start_info.start_time_secs == 12.5
    assert len(pd.session_start_info.group_name) == 64
    hp = tblog.read_hparams(s.SerializeToString())
    assert set(hp) == set(params)
    assert hp["load_factor"] == 1.5 and hp["pingAsObs"] == 0 and hp["agent_type"] == "dqn_buffer"
    assert hp["topology_name"] == "abilene" and isinstance(hp["topology"], str)
    W = tblog.SessionWriters(str(tmp_path / "logs"), hparams=params)
    W.close()
    files = sorted(os.listdir(tmp_path / "logs"))
    tags = [t for f in files if f.startswith("events") for e in tblog.read_events(str(tmp_path / "logs" / f))
            for t, _, _ in e["values"]]
    assert sorted(tags) == ["_hparams_/session_start_info", "custom_scalars__config__"]


def _stream(oracle_mod, topo, params, n):
    """(node, obs, done, info, action) for the first n notifications, SP decisions."""
    o = oracle_mod.OracleSim(topo, params)
    table = sp_next_hop_table(topo)
    ovi = topo.overlay_index
    out, last_done = [], {}
    obs = o.step(-1)
    while obs is not None and len(out) < n:
        v = o.pending_node()
        if int(obs[0]) == 1000:
            a = 0
            out.append((v, [1000], last_done.get(v, False), o.last_info(), a))
        else:
            rec = o.records()[-1]
            done = int(rec["status"]) == 3
            last_done[v] = done
            a = 0 if int(obs[0]) == int(ovi[v]) else int(table[v, topo.overlay_nodes[obs[0]]])
            out.append((v, [int(x) for x in obs[:1 + int(topo.degrees[v])]], done, o.last_info(), a))
        obs = o.step(a)
    return o, out


@pytest.mark.parametrize("train", [0, 1])
def test_agent_stats_against_records(oracle_mod, tmp_path, train):
    topo = Topology.example("abilene", 0, 2.0)                   # drops occur at load 2
    params = engine_params(topo, sim_time_s=3.0, ping_as_obs=1, notify_dest=1, train=train)
    o, stream = _stream(oracle_mod, topo, params, 5000)
    A = tblog.AgentStats({int(v): int(topo.overlay_index[v]) for v in topo.overlay_nodes}, start_time=0.0)
    for v, obs, done, info, a in stream:
        A.observe(v, obs, done, info, a)
    assert A.total_nb_iterations == len(stream)
    n_ctrl = sum(1 for s in stream if s[1] == [1000])
    assert (n_ctrl > 0) == bool(train) and A.small_signaling_pkt_counter == n_ctrl
    # independent recount from the decision records of the same notifications
    recs = o.records()[:A.nb_transitions]
    by_uid = collections.defaultdict(list)
    for r in recs:
        by_uid[int(r["uid"])].append(r)
    dest = [u for u, rs in by_uid.items() if int(rs[-1]["status"]) == 3]
    assert A.total_arrived_pkts == len(dest) > 0
    assert A.total_hops == sum(len(by_uid[u]) - 1 for u in dest)
    assert A.total_new_rcv_pkts == len(by_uid)
    e2e = sum(int(by_uid[u][-1]["t_ns"]) / 1e9 - int(by_uid[u][-1]["start_s"]) for u in dest)
    assert abs(A.total_e2e_delay - e2e) <= 1e-6 * len(dest)
    hop_sum = sum(int(rs[i]["t_ns"]) / 1e9 - int(rs[i - 1]["t_ns"]) / 1e9
                  for rs in by_uid.values() for i in range(1, len(rs)))
    n_transit = sum(len(rs) - 1 for rs in by_uid.values())
    assert abs(A.total_rewards_with_loss - hop_sum) <= 2e-6 * n_transit
    assert A.node_lost_pkts > 0 and A.sim["dropped"] >= A.node_lost_pkts
    # the tag set and step conventions (tb_logger.py:70-140)
    W = tblog.SessionWriters(str(tmp_path / "logs"))
    W.write(A, now=10.0)
    W.close()
    ev = tblog.read_events(W.session.path)[1:]
    assert [e["values"][0][0] for e in ev] == SESSION_TAGS
    it, tt = A.total_nb_iterations, int((A.base_curr_time + A.curr_time) * 1e6)
    got = {e["values"][0][0]: (e["step"], e["values"][0][1]) for e in ev}
    assert got["total_hops_over_iterations"] == (it, A.total_hops)
    assert got["total_hops_over_time"][0] == tt
    lr = A.sim["dropped"] / A.sim["injected"]
    assert got["loss_ratio_over_time"][1] == pytest.approx(lr, rel=1e-6)
    assert got["avg_hops_over_iterations"][1] == pytest.approx(A.total_hops / A.sim["delivered"], rel=1e-6)
    assert got["ma_avg_hops_over_time"][1] == pytest.approx(np.mean(A.nb_hops), rel=1e-6)
    assert got["sim_second_per_real_seconds"][1] == pytest.approx(10.0 / A.curr_time, rel=1e-6)
    for wr, key in ((W.arrived, "delivered"), (W.lost, "dropped"), (W.new, "injected")):
        e = tblog.read_events(wr.path)[1:]
        assert [(x["values"][0][0], x["step"], x["values"][0][1]) for x in e] == [
            ("pkts_over_iterations", it, A.sim[key]), ("pkts_over_time", tt, A.sim[key])]
    par = tblog.read_events(W.parent.path)
    assert par[1]["values"][0][0] == "custom_scalars__config__" and par[1]["step"] == 0
    # test-phase writer (tb_logger.py:142-164)
    p = tblog.stats_writer_test(str(tmp_path / "logs" / "test_results"), A, 2.0, "final")
    e = tblog.read_events(p)[1:]
    assert [x["values"][0][0] for x in e] == TEST_TAGS and {x["step"] for x in e} == {200}
    assert os.path.dirname(p).endswith(os.path.join("test_results", "final"))


@pytest.mark.gpu
def test_agent_stats_from_gpu_session(oracle_mod, tmp_path):
    """The GPU session's notification stream (PrismaSession, one engine replica) gives the
    same AgentStats, hence the same TensorBoard scalars, as the oracle's."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs an MI355X")
    from prisma_amd.ns3env import PrismaSession
    topo = Topology.example("abilene", 0, 2.0)
    kw = dict(sim_time_s=2.0, ping_as_obs=1, train=1)
    _, ref = _stream(oracle_mod, topo, engine_params(topo, notify_dest=1, **kw), 3000)
    ovi = {int(v): int(topo.overlay_index[v]) for v in topo.overlay_nodes}
    A_ref, A_gpu = tblog.AgentStats(ovi, start_time=0.0), tblog.AgentStats(ovi, start_time=0.0)
    for v, obs, done, info, a in ref:
        A_ref.observe(v, obs, done, info, a)
    s = PrismaSession(topo=topo, base_port=7300, **kw)
    table = sp_next_hop_table(topo)
    n = 0
    while s.pending() is not None and n < len(ref):
        v, obs, done, info = s.pending()
        a = 0 if int(obs[0]) in (ovi[v], 1000) else int(table[v, topo.overlay_nodes[obs[0]]])
        A_gpu.observe(v, obs, done, info, a)
        s.apply(a)
        n += 1
    s.close()
    assert n == len(ref)
    for k in ("total_nb_iterations", "nb_transitions", "total_arrived_pkts", "total_hops", "total_e2e_delay",
              "total_rewards_with_loss", "node_lost_pkts", "small_signaling_pkt_counter", "curr_time"):
        assert getattr(A_gpu, k) == getattr(A_ref, k), k
    assert A_gpu.sim == A_ref.sim and A_gpu.delays == A_ref.delays and A_gpu.nb_hops == A_ref.nb_hops
