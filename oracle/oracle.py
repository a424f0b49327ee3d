"""ctypes binding of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg (as the parity checker / CPU baseline), never from the
prisma_amd package.  See oracle/prisma_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "prisma_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


class OrConfig(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_int32), ("n_links", C.c_int32), ("n_flows", C.c_int32), ("max_deg", C.c_int32),
        ("row_ptr", C.POINTER(C.c_int32)), ("link_dst", C.POINTER(C.c_int32)),
        ("link_rev", C.POINTER(C.c_int32)), ("flow_src", C.POINTER(C.c_int32)),
        ("flow_dst", C.POINTER(C.c_int32)), ("flow_rate_bps", C.POINTER(C.c_uint64)),
        ("link_bps", C.c_uint64), ("link_delay_ns", C.c_int64), ("max_buffer_bytes", C.c_uint32),
        ("packet_size", C.c_uint32), ("sim_time_s", C.c_double), ("ping_interval_s", C.c_float),
        ("ma_size", C.c_uint32), ("ping_as_obs", C.c_uint32), ("auto_reset", C.c_uint32),
        ("loss_penalty", C.c_double), ("seed", C.c_uint64), ("replica", C.c_uint32),
        ("episode", C.c_uint32), ("notify_dest", C.c_uint32), ("train", C.c_uint32),
        ("n_overlay", C.c_int32), ("n_tunnels", C.c_int32),
        ("overlay_nodes", C.POINTER(C.c_int32)), ("overlay_index", C.POINTER(C.c_int32)),
        ("ov_row_ptr", C.POINTER(C.c_int32)), ("tun_dst", C.POINTER(C.c_int32)),
        ("tun_link", C.POINTER(C.c_int32)), ("next_link", C.POINTER(C.c_int32)),
        ("signaling_type", C.c_uint32), ("big_signaling", C.c_uint32), ("sync_step_s", C.c_float),
        ("big_signaling_bytes", C.c_uint32), ("rng_mode", C.c_uint32), ("rng_stream_offset", C.c_uint32),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        L.or_create.restype = C.c_void_p
        L.or_create.argtypes = [C.POINTER(OrConfig)]
        L.or_destroy.argtypes = [C.c_void_p]
        L.or_step.restype = C.c_int
        L.or_step.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
        L.or_run_table.restype = C.c_int64
        L.or_run_table.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.or_run_mlp.restype = C.c_int64
        L.or_run_mlp.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.or_mlp_action.restype = C.c_int32
        L.or_mlp_action.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
        L.or_mlp_q.restype = C.c_int32
        L.or_mlp_q.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
        L.or_mlp_q_batch.restype = None
        L.or_mlp_q_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int32,
                                     C.c_void_p, C.c_int32, C.c_void_p]
        L.or_det_expm1.restype = C.c_double
        L.or_det_expm1.argtypes = [C.c_double]
        L.or_det_expm1f.restype = C.c_float
        L.or_det_expm1f.argtypes = [C.c_float]
        L.or_pending_node.restype = C.c_int32
        L.or_pending_node.argtypes = [C.c_void_p]
        L.or_record_count.restype = C.c_int64
        L.or_record_count.argtypes = [C.c_void_p]
        L.or_obs_width.restype = C.c_int32
        L.or_obs_width.argtypes = [C.c_void_p]
        L.or_copy_records.restype = C.c_int64
        L.or_copy_records.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]
        L.or_counters.argtypes = [C.c_void_p, C.c_void_p]
        L.or_diag.argtypes = [C.c_void_p, C.c_void_p]
        L.or_enable_trace.argtypes = [C.c_void_p, C.c_int]
        L.or_trace_count.restype = C.c_int64
        L.or_trace_count.argtypes = [C.c_void_p]
        L.or_copy_trace.restype = C.c_int64
        L.or_copy_trace.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]
        L.or_last_info.restype = C.c_int32
        L.or_last_info.argtypes = [C.c_void_p, C.c_char_p, C.c_int32]
        L.or_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.or_det_log.restype = C.c_double
        L.or_det_log.argtypes = [C.c_double]
        L.or_seconds_to_ns.restype = C.c_int64
        L.or_seconds_to_ns.argtypes = [C.c_double]
        L.or_py_micros.restype = C.c_uint64
        L.or_py_micros.argtypes = [C.c_int64]
        L.or_mrg_pow2.argtypes = [C.c_int, C.POINTER(C.c_uint64)]
        L.or_mrg_first_u01.restype = C.c_double
        L.or_mrg_first_u01.argtypes = [C.c_uint32, C.c_uint64, C.c_uint64]
        _lib = L
    return _lib


def det_expm1(x: float) -> float:
    return float(lib().or_det_expm1(float(x)))


def det_expm1f(x: float) -> float:
    """The fp32 expm1 of the DQN-buffer ELU (x <= 0), as the engine computes it."""
    return float(lib().or_det_expm1f(float(x)))


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().or_philox4x32_10(c, k, o)
    return list(o)


class OracleSim:
    """One replica of the scenario on the CPU (literal heap-based DES)."""

    def __init__(self, topo, params: dict, replica: int = 0, episode: int = 0):
        from prisma_amd.records import record_dtype, COUNTERS_DTYPE  # layout only
        self.topo = topo
        self._keep = []

        def arr(a, ct, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            self._keep.append(a)
            return a.ctypes.data_as(C.POINTER(ct))

        cfg = OrConfig()
        cfg.n_nodes = topo.n_nodes
        cfg.n_links = topo.n_links
        cfg.n_flows = topo.n_flows
        cfg.max_deg = topo.max_deg
        cfg.row_ptr = arr(topo.row_ptr, C.c_int32, np.int32)
        cfg.link_dst = arr(topo.link_dst, C.c_int32, np.int32)
        cfg.link_rev = arr(topo.link_rev, C.c_int32, np.int32)
        cfg.flow_src = arr(topo.flow_src, C.c_int32, np.int32)
        cfg.flow_dst = arr(topo.flow_dst, C.c_int32, np.int32)
        cfg.flow_rate_bps = arr(topo.flow_rate_bps, C.c_uint64, np.uint64)
        cfg.link_bps = int(params["link_bps"])
        cfg.link_delay_ns = int(params["link_delay_ns"])
        cfg.max_buffer_bytes = int(params["max_buffer_bytes"])
        cfg.packet_size = int(params["packet_size"])
        cfg.sim_time_s = float(params["sim_time_s"])
        cfg.ping_interval_s = float(params["ping_interval_s"])
        cfg.ma_size = int(params["ma_size"])
        cfg.ping_as_obs = int(params["ping_as_obs"])
        cfg.auto_reset = 0
        cfg.loss_penalty = float(params["loss_penalty"])
        cfg.seed = int(params["seed"])
        cfg.replica = int(replica)
        cfg.episode = int(episode)
        cfg.notify_dest = int(params.get("notify_dest", 0))
        cfg.train = int(params.get("train", 0))
        cfg.n_overlay = topo.n_overlay
        cfg.n_tunnels = topo.n_tunnels
        cfg.overlay_nodes = arr(topo.overlay_nodes, C.c_int32, np.int32)
        cfg.overlay_index = arr(topo.overlay_index, C.c_int32, np.int32)
        cfg.ov_row_ptr = arr(topo.ov_row_ptr, C.c_int32, np.int32)
        cfg.tun_dst = arr(topo.tun_dst, C.c_int32, np.int32)
        cfg.tun_link = arr(topo.tun_link, C.c_int32, np.int32)
        n = topo.n_nodes
        nl = np.full((n, n), -1, dtype=np.int32)
        for x in range(n):
            for y in range(n):
                if x != y:
                    nl[x, y] = topo.link_id(x, int(topo.next_hop[x, y]))
        cfg.next_link = arr(nl, C.c_int32, np.int32)
        cfg.signaling_type = int(params.get("signaling_type", 0))
        cfg.big_signaling = int(params.get("big_signaling", 0))
        cfg.sync_step_s = float(params.get("sync_step_s", 1.0))
        cfg.big_signaling_bytes = int(params.get("big_signaling_bytes", 512))
        cfg.rng_mode = int(params.get("rng_mode", 0))
        cfg.rng_stream_offset = int(params.get("rng_stream_offset", 0))
        self._cfg = cfg
        self.W = topo.obs_width
        self.rec_dtype = record_dtype(self.W)
        self.cnt_dtype = COUNTERS_DTYPE
        self.h = lib().or_create(C.byref(cfg))

    def close(self):
        if self.h:
            lib().or_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def step(self, action: int = -1):
        obs = np.zeros(self.W, dtype=np.int32)
        r = lib().or_step(self.h, int(action), obs.ctypes.data)
        return (obs if r else None)

    def run_table(self, table: np.ndarray, max_hops: int) -> int:
        t = np.ascontiguousarray(table, dtype=np.uint8)
        return int(lib().or_run_table(self.h, t.ctypes.data, int(max_hops)))

    def records(self, first: int = 0, count: int = None) -> np.ndarray:
        n = int(lib().or_record_count(self.h))
        if count is None:
            count = n - first
        out = np.zeros(max(count, 0), dtype=self.rec_dtype)
        got = lib().or_copy_records(self.h, int(first), int(count), out.ctypes.data)
        return out[:got]

    def counters(self) -> np.ndarray:
        out = np.zeros(1, dtype=self.cnt_dtype)
        lib().or_counters(self.h, out.ctypes.data)
        return out[0]

    def diag(self) -> dict:
        """Test diagnostics (or_diag): drops inside tunnels, FIFO depths now."""
        out = np.zeros(4, dtype=np.int64)
        lib().or_diag(self.h, out.ctypes.data)
        return dict(relay_drops=int(out[0]), max_queue=int(out[1]), queued=int(out[2]), deep_fifos=int(out[3]))

    def enable_trace(self, on: bool = True):
        lib().or_enable_trace(self.h, int(on))

    def trace(self) -> np.ndarray:
        n = int(lib().or_trace_count(self.h))
        out = np.zeros((n, 4), dtype=np.int64)
        lib().or_copy_trace(self.h, 0, n, out.ctypes.data)
        return out

    def run_mlp(self, weights: np.ndarray, max_hops: int) -> int:
        w = np.ascontiguousarray(weights, dtype=np.float32)
        return int(lib().or_run_mlp(self.h, w.ctypes.data, int(max_hops)))

    def mlp_action(self, weights: np.ndarray, node: int, obs) -> int:
        w = np.ascontiguousarray(weights, dtype=np.float32)
        o = np.ascontiguousarray(obs, dtype=np.uint32)
        return int(lib().or_mlp_action(self.h, w.ctypes.data, int(node), o.ctypes.data))

    def mlp_q(self, weights: np.ndarray, node: int, obs) -> np.ndarray:
        """The restatement's fixed-order fp32 Q values (length = the node's degree)."""
        w = np.ascontiguousarray(weights, dtype=np.float32)
        o = np.ascontiguousarray(obs, dtype=np.uint32)
        q = np.zeros(max(self.topo.max_deg, 1), dtype=np.float32)
        lib().or_mlp_q(self.h, w.ctypes.data, int(node), o.ctypes.data, q.ctypes.data)
        return q[:int(self.topo.degrees[node])]

    def mlp_q_batch(self, weights: np.ndarray, nodes, obs):
        """(Q [n, max_deg] with +inf past each node's degree, actions [n]) of the restatement."""
        w = np.ascontiguousarray(weights, dtype=np.float32)
        nd = np.ascontiguousarray(nodes, dtype=np.int32)
        o = np.ascontiguousarray(obs, dtype=np.uint32)
        D = max(self.topo.max_deg, 1)
        q = np.full((nd.size, D), np.inf, dtype=np.float32)
        a = np.zeros(nd.size, dtype=np.int32)
        lib().or_mlp_q_batch(self.h, w.ctypes.data, nd.size, nd.ctypes.data, o.ctypes.data, o.shape[1],
                             q.ctypes.data, D, a.ctypes.data)
        return q, a

    def pending_node(self) -> int:
        return int(lib().or_pending_node(self.h))

    def last_info(self) -> str:
        buf = C.create_string_buffer(8192)
        lib().or_last_info(self.h, buf, 8192)
        return buf.value.decode()
