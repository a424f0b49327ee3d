"""TensorBoard logging of a PRISMA session without TensorFlow.

The reference logs through ``tf.summary`` (prisma/source/tb_logger.py:15-164, called from
prisma/main.py:71-90,145,180).  This module writes the same runs, tags and steps as
TensorBoard event files:

* ``EventFileWriter`` — TFRecord framing (length, masked CRC-32C of the length, payload,
  masked CRC-32C of the payload) of ``Event`` protobufs.  The first record carries
  ``file_version = "brain.Event:2"``; scalars are TF2-style tensor summaries
  (``tensor {dtype: DT_FLOAT, tensor_shape {}, tensor_content: <4 bytes>}`` with
  ``plugin_name: "scalars"`` metadata), what ``tf.summary.scalar`` writes.
* ``AgentStats`` — the Agent class variables tb_logger reads, restated from the
  Forwarder's bookkeeping over the notification stream (forwarder.py:197-289 treat_info,
  :291-332 run, :334-431 handle_new_packet / handle_transit_packet / handle_done).
* ``stats_writer_train`` / ``stats_writer_test`` / ``custom_plots`` — tb_logger.py's three
  functions with the same tags, writers and step conventions.

The protobuf messages are declared from a descriptor (``protoc`` and TensorFlow are not
installed); field numbers follow tensorflow/core/util/event.proto,
tensorflow/core/framework/{summary,tensor,tensor_shape,types}.proto and
tensorboard/plugins/custom_scalar/layout.proto.  A real TensorBoard reading these files is
unverified here (not installed): the tests pin the framing (CRC-32C check value), the
round trip and the tag set / values against the reference's formulas.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory, struct_pb2

F = descriptor_pb2.FieldDescriptorProto

DT_FLOAT, DT_STRING = 1, 7
DATA_CLASS_SCALAR = 1
FILE_VERSION = "brain.Event:2"
CUSTOM_SCALARS_TAG = "custom_scalars__config__"
HPARAMS_TAG = "_hparams_/session_start_info"       # tensorboard/plugins/hparams/metadata.py


def _file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="prisma_amd/tb_event.proto", package="tensorflow", syntax="proto3")
    R, O = F.LABEL_REPEATED, F.LABEL_OPTIONAL

    def msg(name, fields, parent=None):
        m = (parent.nested_type if parent is not None else fd.message_type).add(name=name)
        for num, fname, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
        return m

    msg("TensorShapeProto", [(2, "dim", F.TYPE_MESSAGE, R, ".tensorflow.TensorShapeProto.Dim"),
                             (3, "unknown_rank", F.TYPE_BOOL, O, None)])
    msg("Dim", [(1, "size", F.TYPE_INT64, O, None), (2, "name", F.TYPE_STRING, O, None)],
        parent=fd.message_type[-1])
    msg("TensorProto", [(1, "dtype", F.TYPE_INT32, O, None),        # enum DataType (DT_FLOAT 1, DT_STRING 7)
                        (2, "tensor_shape", F.TYPE_MESSAGE, O, ".tensorflow.TensorShapeProto"),
                        (3, "version_number", F.TYPE_INT32, O, None),
                        (4, "tensor_content", F.TYPE_BYTES, O, None),
                        (5, "float_val", F.TYPE_FLOAT, R, None),
                        (8, "string_val", F.TYPE_BYTES, R, None)])
    sm = msg("SummaryMetadata", [(1, "plugin_data", F.TYPE_MESSAGE, O, ".tensorflow.SummaryMetadata.PluginData"),
                                 (2, "display_name", F.TYPE_STRING, O, None),
                                 (3, "summary_description", F.TYPE_STRING, O, None),
                                 (4, "data_class", F.TYPE_INT32, O, None)])   # enum DataClass
    msg("PluginData", [(1, "plugin_name", F.TYPE_STRING, O, None), (2, "content", F.TYPE_BYTES, O, None)], parent=sm)
    s = msg("Summary", [(1, "value", F.TYPE_MESSAGE, R, ".tensorflow.Summary.Value")])
    msg("Value", [(7, "node_name", F.TYPE_STRING, O, None), (1, "tag", F.TYPE_STRING, O, None),
                  (9, "metadata", F.TYPE_MESSAGE, O, ".tensorflow.SummaryMetadata"),
                  (2, "simple_value", F.TYPE_FLOAT, O, None),
                  (8, "tensor", F.TYPE_MESSAGE, O, ".tensorflow.TensorProto")], parent=s)
    msg("Event", [(1, "wall_time", F.TYPE_DOUBLE, O, None), (2, "step", F.TYPE_INT64, O, None),
                  (3, "file_version", F.TYPE_STRING, O, None), (5, "summary", F.TYPE_MESSAGE, O, ".tensorflow.Summary")])
    # tensorboard/plugins/custom_scalar/layout.proto
    msg("MultilineChartContent", [(1, "tag", F.TYPE_STRING, R, None)])
    msg("Chart", [(1, "title", F.TYPE_STRING, O, None),
                  (2, "multiline", F.TYPE_MESSAGE, O, ".tensorflow.MultilineChartContent")])
    msg("Category", [(1, "title", F.TYPE_STRING, O, None), (2, "chart", F.TYPE_MESSAGE, R, ".tensorflow.Chart"),
                     (3, "closed", F.TYPE_BOOL, O, None)])
    msg("Layout", [(1, "version", F.TYPE_INT32, O, None), (2, "category", F.TYPE_MESSAGE, R, ".tensorflow.Category")])
    # tensorboard/plugins/hparams/plugin_data.proto (the session_start_info arm of HParamsPluginData)
    fd.dependency.append("google/protobuf/struct.proto")
    ssi = msg("SessionStartInfo", [(1, "hparams", F.TYPE_MESSAGE, R, ".tensorflow.SessionStartInfo.HparamsEntry"),
                                   (2, "model_uri", F.TYPE_STRING, O, None),
                                   (3, "monitor_url", F.TYPE_STRING, O, None),
                                   (4, "group_name", F.TYPE_STRING, O, None),
                                   (5, "start_time_secs", F.TYPE_DOUBLE, O, None)])
    ent = msg("HparamsEntry", [(1, "key", F.TYPE_STRING, O, None),
                               (2, "value", F.TYPE_MESSAGE, O, ".google.protobuf.Value")], parent=ssi)
    ent.options.map_entry = True
    msg("HParamsPluginData", [(1, "version", F.TYPE_INT32, O, None),
                              (3, "session_start_info", F.TYPE_MESSAGE, O, ".tensorflow.SessionStartInfo")])
    return fd


_pool = descriptor_pool.DescriptorPool()
_pool.AddSerializedFile(struct_pb2.DESCRIPTOR.serialized_pb)
_pool.AddSerializedFile(_file().SerializeToString())
_classes = message_factory.GetMessages([_file()], pool=_pool)
Event = _classes["tensorflow.Event"]
Summary = _classes["tensorflow.Summary"]
Layout = _classes["tensorflow.Layout"]
HParamsPluginData = _classes["tensorflow.HParamsPluginData"]


# ---------------------------------------------------------------------------
# TFRecord framing
# ---------------------------------------------------------------------------
def _crc32c_table() -> List[int]:
    poly, t = 0x82F63B78, []                      # Castagnoli, reflected
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        t.append(c)
    return t


_CRC_T = _crc32c_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_T[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def tfrecord(payload: bytes) -> bytes:
    n = struct.pack("<Q", len(payload))
    return n + struct.pack("<I", masked_crc32c(n)) + payload + struct.pack("<I", masked_crc32c(payload))


def read_tfrecords(path: str) -> List[bytes]:
    """Payloads of a TFRecord file; raises ValueError on a CRC mismatch or a truncated record."""
    out, buf = [], open(path, "rb").read()
    i = 0
    while i < len(buf):
        if i + 12 > len(buf):
            raise ValueError("truncated record header")
        n = buf[i:i + 8]
        (ln,) = struct.unpack("<Q", n)
        if struct.unpack("<I", buf[i + 8:i + 12])[0] != masked_crc32c(n):
            raise ValueError("length CRC mismatch")
        p = buf[i + 12:i + 12 + ln]
        if len(p) != ln or struct.unpack("<I", buf[i + 12 + ln:i + 16 + ln])[0] != masked_crc32c(p):
            raise ValueError("payload CRC mismatch")
        out.append(p)
        i += 16 + ln
    return out


def read_events(path: str) -> List[dict]:
    """Decoded events: {"wall_time", "step", "file_version", "values": [(tag, value, plugin)]}; scalar
    tensor summaries decode to float, string tensors to bytes."""
    evs = []
    for p in read_tfrecords(path):
        e = Event.FromString(p)
        vals = []
        for v in e.summary.value:
            t = v.tensor
            if t.dtype == DT_FLOAT and len(t.tensor_content) == 4:
                x = struct.unpack("<f", t.tensor_content)[0]
            elif t.dtype == DT_FLOAT and len(t.float_val):
                x = float(t.float_val[0])
            elif t.dtype == DT_STRING and len(t.string_val):
                x = bytes(t.string_val[0])
            else:
                x = float(v.simple_value)
            vals.append((v.tag, x, v.metadata.plugin_data.plugin_name))
        evs.append({"wall_time": e.wall_time, "step": e.step, "file_version": e.file_version, "values": vals})
    return evs


class EventFileWriter:
    """``tf.summary.create_file_writer(logdir)``: one events file per writer, named like TF2's
    (events.out.tfevents.<secs>.<host>.<pid>.<n>.v2)."""
    _n = 0

    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        EventFileWriter._n += 1
        self.path = os.path.join(logdir, "events.out.tfevents.%d.%s.%d.%d.v2" % (
            int(time.time()), socket.gethostname(), os.getpid(), EventFileWriter._n))
        self._f = open(self.path, "wb")
        self._write(Event(wall_time=time.time(), file_version=FILE_VERSION))

    def _write(self, ev) -> None:
        self._f.write(tfrecord(ev.SerializeToString()))

    def scalar(self, tag: str, value: float, step: int) -> None:
        """tf.summary.scalar: a float32 scalar tensor summary (scalars plugin)."""
        ev = Event(wall_time=time.time(), step=int(step))
        v = ev.summary.value.add(tag=tag)
        v.metadata.plugin_data.plugin_name = "scalars"
        v.metadata.data_class = DATA_CLASS_SCALAR
        v.tensor.dtype = DT_FLOAT
        v.tensor.tensor_shape.SetInParent()
        v.tensor.tensor_content = struct.pack("<f", float(np.float32(value)))
        self._write(ev)

    def raw_summary(self, summary_bytes: bytes, step: int) -> None:
        """tf.summary.experimental.write_raw_pb."""
        ev = Event(wall_time=time.time(), step=int(step))
        ev.summary.MergeFromString(summary_bytes)
        self._write(ev)

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        if not self._f.closed:
            self._f.close()


# ---------------------------------------------------------------------------
# the Agent statistics tb_logger reads (forwarder.py bookkeeping)
# ---------------------------------------------------------------------------
def _tok(tokens: Sequence[str], i: int) -> str:
    return tokens[i].split("=")[-1]


class AgentStats:
    """Agent class variables after the Forwarder threads consumed a notification stream.

    ``observe(node, obs, done, info)`` takes the notifications in the order the simulator
    emits them (one REQ/REP exchange at a time, so this is also the order the reference's
    threads process them), each as ``Ns3Env.step`` returns it.  Only the statistics are
    kept: replay buffers, learning and exploration are the trainer's (prisma_amd/trainer.py).
    """

    def __init__(self, overlay_index: Dict[int, int], start_time: Optional[float] = None):
        self.ovi = dict(overlay_index)             # node -> its own overlay index (Forwarder.index)
        self.start_time = time.time() if start_time is None else start_time
        self.base_curr_time = 0.0
        self.curr_time = 0.0
        self.total_nb_iterations = 0
        self.nb_transitions = 0
        self.total_new_rcv_pkts = 0
        self.total_arrived_pkts = 0
        self.total_hops = 0
        self.total_e2e_delay = 0.0
        self.total_rewards_with_loss = 0.0
        self.node_lost_pkts = 0
        self.small_signaling_overhead_counter = 0.0
        self.small_signaling_pkt_counter = 0
        self.delays: List[float] = []
        self.nb_hops: List[int] = []
        self.rewards: List[float] = []
        self.temp_obs: Dict[int, dict] = {}
        self.pkt_tracking: Dict[int, dict] = {}
        self.transition_number: Dict[int, int] = {v: 0 for v in self.ovi}
        self.sim = dict(avg_e2e_delay=0.0, cost=0.0, global_avg_e2e_delay=0.0, global_cost=0.0,
                        dropped=0.0, delivered=0.0, injected=0.0, buffered=0.0, global_dropped=0.0,
                        global_delivered=0.0, global_injected=0.0, global_buffered=0.0, signaling_overhead=0.0)

    def _treat_info(self, info: str) -> tuple:
        """forwarder.py:197-289: returns (is_control, delay_time, pkt_id)."""
        t = info.split(",")
        delay_time = float(_tok(t, 0))
        pkt_size = float(_tok(t, 1))
        self.curr_time = float(_tok(t, 2))
        pkt_id = int(_tok(t, 3))
        ptype = int(_tok(t, 4))
        if ptype == 0:
            for lid in _tok(t, 18).split(";")[:-1]:
                if self.temp_obs.get(int(lid)) is None:
                    continue                                   # the reference prints "error"
                self.node_lost_pkts += 1
                self.pkt_tracking.pop(int(lid), None)
        else:
            if ptype == 2:
                self.small_signaling_overhead_counter += pkt_size
                self.small_signaling_pkt_counter += 1
            return True, delay_time, pkt_id
        s = self.sim
        s["avg_e2e_delay"] = float(_tok(t, 5))
        s["cost"] = float(_tok(t, 6))
        s["global_avg_e2e_delay"] = float(_tok(t, 7))
        s["global_cost"] = float(_tok(t, 8))
        s["dropped"] = float(_tok(t, 9))
        s["delivered"] = float(_tok(t, 10))
        s["injected"] = float(_tok(t, 11))
        s["buffered"] = float(_tok(t, 12))
        t13 = float(_tok(t, 13))
        s["global_dropped"] = t13 + s["dropped"]
        s["global_delivered"] = float(_tok(t, 14)) + s["delivered"]
        s["global_injected"] = float(_tok(t, 15)) + s["injected"]
        s["global_buffered"] = float(_tok(t, 16)) + s["buffered"]
        s["signaling_overhead"] = float(_tok(t, 17))
        if s["global_delivered"] > 0:                          # forwarder.py:283-284, literally
            s["global_avg_e2e_delay"] = ((s["global_avg_e2e_delay"] * t13)
                                         + (s["avg_e2e_delay"] * s["delivered"])) / s["global_delivered"]
        if s["global_delivered"] + s["global_dropped"] > 0:   # :285-286 (token 13 twice, as there)
            s["global_cost"] = ((s["global_cost"] * (t13 + t13)) + (s["cost"] * (s["dropped"] + s["delivered"]))
                                ) / (s["global_dropped"] + s["global_delivered"])
        return False, delay_time, pkt_id

    def observe(self, node: int, obs: Sequence[int], done: bool, info: str, action: int = 0) -> None:
        """One notification at `node`; `action` is the one the node's agent then applies
        (only used for the next hop's bookkeeping, as Agent.temp_obs)."""
        if done and int(obs[0]) == -1:                          # end of episode (forwarder.py:304)
            return
        self.transition_number[node] = self.transition_number.get(node, 0) + 1
        self.total_nb_iterations += 1
        control, delay_time, pkt_id = self._treat_info(info)
        if control:
            return
        self.nb_transitions += 1
        me = self.ovi[node]
        if pkt_id not in self.pkt_tracking:                     # handle_new_packet
            self.total_new_rcv_pkts += 1
            self.pkt_tracking[pkt_id] = {"hops": [me]}
        else:                                                   # handle_transit_packet
            st = self.temp_obs.pop(pkt_id)
            hop_time_real = self.curr_time - st["time"]
            self.total_rewards_with_loss += hop_time_real
            self.pkt_tracking[pkt_id]["hops"].append(me)
            self.rewards.append(hop_time_real)
            if done:                                            # handle_done
                self.total_arrived_pkts += 1
                hops = len(self.pkt_tracking[pkt_id]["hops"]) - 1
                self.total_hops += hops
                self.total_e2e_delay += delay_time
                self.delays.append(delay_time)
                self.nb_hops.append(hops)
                self.nb_hops = self.nb_hops[-50:]
                self.delays = self.delays[-50:]
                self.pkt_tracking.pop(pkt_id)
        # Forwarder.step on this obs (forwarder.py:149-160): a decision is recorded unless
        # the packet is at its destination or this is the node's first transition
        if int(obs[0]) != me and int(obs[0]) not in (-1, 1000) and self.transition_number[node] >= 1:
            self.temp_obs[pkt_id] = {"time": self.curr_time, "action": int(action), "obs": list(obs)}

    def end_episode(self) -> None:
        """main.py:176: base_curr_time accumulates the episode's simulated time."""
        self.base_curr_time += self.curr_time


# ---------------------------------------------------------------------------
# tb_logger.py
# ---------------------------------------------------------------------------
def custom_plots() -> bytes:
    """tb_logger.py:15-68: the custom-scalars layout summary (tag custom_scalars__config__)."""
    lay = Layout()
    for title, charts in (("Main evaluation metrics", [("Avg Delay per arrived pkts", r"avg_delay_over_time"),
                                                       ("Avg Cost per arrived pkts", r"avg_cost_over_time"),
                                                       ("Loss Ratio", r"loss_ratio_over_time")]),
                          ("Training metrics", [("Td error", r"MSE_loss_over_time"),
                                                ("exploration value", r"exploaration_value_over_time"),
                                                ("replay buffers length", r"replay_buffer_length_over_time")])):
        cat = lay.category.add(title=title)
        for ct, tag in charts:
            ch = cat.chart.add(title=ct)
            ch.multiline.tag.append(tag)
    s = Summary()
    v = s.value.add(tag=CUSTOM_SCALARS_TAG)
    v.metadata.plugin_data.plugin_name = "custom_scalars"
    v.tensor.dtype = DT_STRING
    v.tensor.tensor_shape.SetInParent()
    v.tensor.string_val.append(lay.SerializeToString())
    return s.SerializeToString()


def hparams_summary(params: dict, start_time_secs: Optional[float] = None, trial_id: Optional[str] = None) -> bytes:
    """main.py:79-85 (``hp.hparams(dict_to_store)``): the session's parameters as the hparams
    plugin's session-start summary (tag ``_hparams_/session_start_info``, plugin ``hparams``,
    content = HParamsPluginData{version 0, session_start_info}), restated from TensorBoard's
    hparams summary_v2 API: values go in by type (bool, then int/float as number_value, str);
    the group name is the trial id, or the SHA-256 of the sorted-key JSON of the hparams.
    main.py first turns the non-scalar entries (G, load_path, simArgs) into strings; this does
    the same for any value that is not bool/int/float/str.  Parity unpinned: TensorFlow and
    TensorBoard are not installed here, so no reference-written file could be compared."""
    import hashlib
    import json
    hps = {}
    for k, v in params.items():
        if isinstance(v, (np.bool_,)):
            v = bool(v)
        elif isinstance(v, (np.integer, np.floating)):
            v = v.item()
        elif v is None or not isinstance(v, (bool, int, float, str)):
            v = str(v)
        hps[str(k)] = v
    pd = HParamsPluginData(version=0)
    si = pd.session_start_info
    si.start_time_secs = time.time() if start_time_secs is None else float(start_time_secs)
    si.group_name = trial_id if trial_id is not None else hashlib.sha256(
        json.dumps(hps, sort_keys=True).encode("utf-8")).hexdigest()
    for k in sorted(hps):
        v = hps[k]
        if isinstance(v, bool):
            si.hparams[k].bool_value = v
        elif isinstance(v, (int, float)):
            si.hparams[k].number_value = float(v)
        else:
            si.hparams[k].string_value = v
    s = Summary()
    val = s.value.add(tag=HPARAMS_TAG)
    val.metadata.plugin_data.plugin_name = "hparams"
    val.metadata.plugin_data.content = pd.SerializeToString()
    val.tensor.dtype = DT_FLOAT
    val.tensor.tensor_shape.SetInParent()
    return s.SerializeToString()


def read_hparams(summary_bytes: bytes) -> dict:
    """Inverse of hparams_summary for tests: {name: value} of the session-start info."""
    s = Summary.FromString(summary_bytes)
    v = [x for x in s.value if x.tag == HPARAMS_TAG][0]
    pd = HParamsPluginData.FromString(v.metadata.plugin_data.content)
    out = {}
    for k, val in pd.session_start_info.hparams.items():
        kind = val.WhichOneof("kind")
        out[k] = getattr(val, kind)
    return out


def _mean(x: List[float]) -> float:
    return float(np.mean(np.array(x, dtype=np.float64))) if len(x) else float("nan")


def stats_writer_train(w_session: EventFileWriter, w_arrived: EventFileWriter, w_lost: EventFileWriter,
                       w_new: EventFileWriter, A: AgentStats, now: Optional[float] = None) -> None:
    """tb_logger.py:70-140 with the same tags and steps (iterations / simulated microseconds)."""
    s = A.sim
    loss_ratio = s["dropped"] / s["injected"] if s["injected"] > 0 else -1
    if s["delivered"] > 0:
        avg_delay, avg_cost, avg_hops = s["avg_e2e_delay"], s["cost"], A.total_hops / s["delivered"]
    else:
        avg_delay = avg_cost = avg_hops = -1
    it = A.total_nb_iterations
    tt = int((A.base_curr_time + A.curr_time) * 1e6)
    now = time.time() if now is None else now
    w = w_session
    w.scalar("total_e2e_delay_over_iterations", A.total_e2e_delay, it)
    w.scalar("total_e2e_delay_over_time", A.total_e2e_delay, tt)
    w.scalar("total_rewards_with_loss_over_iterations", A.total_rewards_with_loss, it)
    w.scalar("total_rewards_with_loss_over_time", A.total_rewards_with_loss, tt)
    w.scalar("loss_ratio_over_time", loss_ratio, tt)
    w.scalar("loss_ratio_over_iterations", loss_ratio, it)
    w.scalar("total_hops_over_iterations", A.total_hops, it)
    w.scalar("total_hops_over_time", A.total_hops, tt)
    w.scalar("avg_hops_over_iterations", avg_hops, it)
    w.scalar("avg_hops_over_time", avg_hops, tt)
    w.scalar("ma_avg_hops_over_iterations", _mean(A.nb_hops), it)
    w.scalar("ma_avg_hops_over_time", _mean(A.nb_hops), tt)
    w.scalar("nb_buffered_pkts_over_time", s["buffered"], tt)
    w.scalar("nb_buffered_pkts_over_iterations", s["buffered"], it)
    w.scalar("signalling ratio", s["signaling_overhead"], tt)
    w.scalar("avg_cost_over_iterations", avg_cost, it)
    w.scalar("avg_cost_over_time", avg_cost, tt)
    w.scalar("avg_delay_over_iterations", avg_delay, it)
    w.scalar("avg_delay_over_time", avg_delay, tt)
    w.scalar("ma_delays_over_iterations", _mean(A.delays), it)
    w.scalar("ma_delays_over_time", _mean(A.delays), tt)
    sim_t = A.base_curr_time + A.curr_time
    w.scalar("sim_second_per_real_seconds", (now - A.start_time) / sim_t if sim_t else float("inf"), tt)
    for wr, val in ((w_arrived, s["delivered"]), (w_lost, s["dropped"]), (w_new, s["injected"])):
        wr.scalar("pkts_over_iterations", val, it)
        wr.scalar("pkts_over_time", val, tt)
    for wr in (w_session, w_arrived, w_lost, w_new):
        wr.flush()


def trainer_stats_writer(w: EventFileWriter, trainer, step: int) -> None:
    """The trainer's own counters (QRoutingTrainer.stats(): signalling overheads, stored weight
    generations, stale_syncs) under a "trainer/" prefix -- not tags of the reference's tb_logger."""
    for k, v in trainer.stats().items():
        w.scalar(f"trainer/{k}", float(v), step)
    w.flush()


def stats_writer_test(results_path: str, A: AgentStats, load_factor: float, model_version: str) -> str:
    """tb_logger.py:142-164: one writer under <results_path>/<model_version>, step = int(100 * load factor).
    Returns the events file path."""
    w = EventFileWriter(os.path.join(results_path, model_version))
    s = A.sim
    step = int(load_factor * 100)
    w.scalar("test_global_injected_pkts", s["global_injected"], step)
    w.scalar("test_overlay_injected_pkts", s["injected"], step)
    w.scalar("test_global_lost_pkts", s["global_dropped"], step)
    w.scalar("test_overlay_lost_pkts", s["dropped"], step)
    w.scalar("test_global_arrived_pkts", s["global_delivered"], step)
    w.scalar("test_overlay_arrived_pkts", s["delivered"], step)
    # the reference swaps the two e2e tags (tb_logger.py:157-158): kept as is
    w.scalar("test_global_e2e_delay", s["avg_e2e_delay"], step)
    w.scalar("test_overlay_e2e_delay", s["global_avg_e2e_delay"], step)
    w.scalar("test_global_loss_rate", s["global_dropped"] / s["global_injected"], step)
    w.scalar("test_overlay_loss_rate", s["dropped"] / s["injected"], step)
    w.scalar("test_global_cost", s["global_cost"], step)
    w.scalar("test_overlay_cost", s["cost"], step)
    w.close()
    return w.path


class SessionWriters:
    """main.py:71-90: the parent, session and nb_{arrived,new,lost}_pkts writers, with the
    session's hparams record (when given) and the custom-scalars layout written once at step 0.  Directory names follow
    argument_parser.py's logs layout (<logs_folder>/stats, /nb_arrived_pkts, ...)."""

    def __init__(self, logs_folder: str, hparams: Optional[dict] = None):
        self.parent = EventFileWriter(logs_folder)
        if hparams is not None:                     # main.py:79-85, a writer of its own on logs_folder
            hw = EventFileWriter(logs_folder)
            hw.raw_summary(hparams_summary(hparams), step=0)
            hw.close()
        self.session = EventFileWriter(os.path.join(logs_folder, "stats"))
        self.arrived = EventFileWriter(os.path.join(logs_folder, "nb_arrived_pkts"))
        self.new = EventFileWriter(os.path.join(logs_folder, "nb_new_pkts"))
        self.lost = EventFileWriter(os.path.join(logs_folder, "nb_lost_pkts"))
        self.parent.raw_summary(custom_plots(), step=0)
        self.parent.flush()

    def write(self, A: AgentStats, now: Optional[float] = None) -> None:
        stats_writer_train(self.session, self.arrived, self.lost, self.new, A, now=now)

    def close(self) -> None:
        for w in (self.parent, self.session, self.arrived, self.new, self.lost):
            w.close()
