"""ctypes binding of libprisma_amd.so (include/prisma.h) on torch HIP memory.

The library is the product: every simulation step runs in its gfx950
kernels.  There is no CPU fallback — if the shared library is missing or no
gfx950 device is present, construction raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from . import buildid
from .records import COUNTERS_DTYPE, record_dtype
from .topology import Topology

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprisma_amd.so")

ABI_VERSION = 10
PRISMA_POLICY_TABLE = 1
PRISMA_POLICY_DQN_BUFFER = 2
PRISMA_ENGINE_AUTO, PRISMA_ENGINE_REGISTER, PRISMA_ENGINE_MEMORY = 0, 1, 2


def dqn_buffer_floats(n: int, d: int) -> int:
    """Length of the packed DQN-buffer weights (include/prisma.h PRISMA_POLICY_DQN_BUFFER)."""
    return n * n * 32 + n * 32 + n * d * 32 + n * 32 + 2 * (n * 64 * 64 + n * 64) + n * 64 * d + n * d


class PrismaError(RuntimeError):
    pass


class _Topo(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_int32), ("n_links", C.c_int32), ("n_flows", C.c_int32), ("max_deg", C.c_int32),
        ("row_ptr", C.c_void_p), ("link_dst", C.c_void_p), ("link_rev", C.c_void_p),
        ("flow_src", C.c_void_p), ("flow_dst", C.c_void_p), ("flow_rate_bps", C.c_void_p),
        ("n_overlay", C.c_int32), ("overlay_nodes", C.c_void_p), ("overlay_adj", C.c_void_p),
    ]


class _Params(C.Structure):
    _fields_ = [
        ("link_bps", C.c_uint64), ("link_delay_ns", C.c_int64), ("max_buffer_bytes", C.c_uint32),
        ("packet_size", C.c_uint32), ("sim_time_s", C.c_double), ("ping_interval_s", C.c_float),
        ("ma_size", C.c_uint32), ("ping_as_obs", C.c_uint32), ("auto_reset", C.c_uint32),
        ("loss_penalty", C.c_double), ("seed", C.c_uint64), ("replica_base", C.c_uint32),
        ("log_capacity", C.c_uint32), ("notify_dest", C.c_uint32), ("train", C.c_uint32),
        ("engine", C.c_uint32), ("signaling_type", C.c_uint32), ("big_signaling", C.c_uint32),
        ("sync_step_s", C.c_float), ("big_signaling_bytes", C.c_uint32),
        ("rng_mode", C.c_uint32), ("rng_stream_offset", C.c_uint32),
    ]


# the defaults of config.engine_params (argument_parser.py:72-74, 86; bigSignalingSize 512)
_PARAM_DEFAULTS = dict(engine=0, signaling_type=0, big_signaling=0, sync_step_s=1.0, big_signaling_bytes=512,
                       rng_mode=0, rng_stream_offset=0)


class _LogView(C.Structure):
    _fields_ = [("records", C.c_void_p), ("record_bytes", C.c_uint32), ("log_capacity", C.c_uint32),
                ("obs_width", C.c_int32), ("n_replicas", C.c_int32)]


class _KernelInfo(C.Structure):
    _fields_ = [("engine", C.c_uint32), ("flow_slots", C.c_int32), ("link_slots", C.c_int32),
                ("tunnels", C.c_uint32), ("ctrl", C.c_uint32), ("relay_ip", C.c_uint32),
                ("relay_dec_bits", C.c_uint32)]


class _Plan(C.Structure):
    _fields_ = [("state_bytes", C.c_uint32), ("lds_bytes", C.c_uint32), ("lds_state_bytes", C.c_uint32),
                ("ring_entries", C.c_uint32), ("record_bytes", C.c_uint32), ("obs_width", C.c_int32),
                ("flow_slots", C.c_int32), ("link_slots", C.c_int32), ("engine", C.c_uint32)]


EXPORTS = [
    "prisma_abi_version", "prisma_last_error", "prisma_build_id", "prisma_create", "prisma_reset", "prisma_step", "prisma_run",
    "prisma_read_counters", "prisma_counters_device", "prisma_log_view", "prisma_copy_log",
    "prisma_copy_counters", "prisma_gather_records", "prisma_state_bytes", "prisma_plan", "prisma_destroy",
    "prisma_compact_pending", "prisma_expand_actions", "prisma_kernel_info",
]

_lib = None


def load_library(path: str = None):
    """Load libprisma_amd.so and declare its C-ABI (raises if absent).

    PRISMA_LIB overrides the path (diagnostic builds, e.g. scripts/ablate.sh).  The default
    library must carry the build id of the sources beside it (prisma_amd/buildid.py): a stale
    binary raises instead of running."""
    global _lib
    if _lib is not None:
        return _lib
    override = path or os.environ.get("PRISMA_LIB")
    path = override or LIB_PATH
    if not os.path.exists(path):
        raise PrismaError(f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(path)
    L.prisma_abi_version.restype = C.c_int
    L.prisma_last_error.restype = C.c_char_p
    L.prisma_build_id.restype = C.c_char_p
    if not override and buildid.sources_present():
        want, got = buildid.source_hash(), L.prisma_build_id().decode()
        if got != want:
            raise PrismaError(f"{path} was built from other sources (build id {got}, sources {want}): "
                              f"rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
    L.prisma_create.restype = C.c_int
    L.prisma_create.argtypes = [C.POINTER(_Topo), C.POINTER(_Params), C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]
    L.prisma_reset.restype = C.c_int
    L.prisma_reset.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    L.prisma_step.restype = C.c_int
    L.prisma_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.prisma_run.restype = C.c_int
    L.prisma_run.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]
    L.prisma_read_counters.restype = C.c_int
    L.prisma_read_counters.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.prisma_counters_device.restype = C.c_int
    L.prisma_counters_device.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    L.prisma_log_view.restype = C.c_int
    L.prisma_log_view.argtypes = [C.c_void_p, C.POINTER(_LogView)]
    L.prisma_copy_log.restype = C.c_int
    L.prisma_copy_log.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
    L.prisma_copy_counters.restype = C.c_int
    L.prisma_copy_counters.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.prisma_gather_records.restype = C.c_int
    L.prisma_gather_records.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
    L.prisma_compact_pending.restype = C.c_int
    L.prisma_compact_pending.argtypes = [C.c_void_p] + [C.c_void_p] * 7 + [C.c_void_p]
    L.prisma_expand_actions.restype = C.c_int
    L.prisma_expand_actions.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p,
                                        C.c_void_p]
    L.prisma_kernel_info.restype = C.c_int
    L.prisma_kernel_info.argtypes = [C.c_void_p, C.POINTER(_KernelInfo)]
    L.prisma_state_bytes.restype = C.c_int
    L.prisma_state_bytes.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.prisma_plan.restype = C.c_int
    L.prisma_plan.argtypes = [C.POINTER(_Topo), C.POINTER(_Params), C.POINTER(_Plan)]
    L.prisma_destroy.restype = None
    L.prisma_destroy.argtypes = [C.c_void_p]
    if L.prisma_abi_version() != ABI_VERSION:
        raise PrismaError("libprisma_amd ABI version mismatch")
    _lib = L
    return L


def build_id() -> str:
    """Build id of the loaded library (prisma_build_id())."""
    return load_library().prisma_build_id().decode()


def _check(rc: int):
    if rc != 0:
        msg = _lib.prisma_last_error().decode(errors="replace")
        raise PrismaError(f"prisma error {rc}: {msg}")


def _stream_handle(stream) -> Optional[int]:
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def _topo_struct(topo: Topology):
    keep = [np.ascontiguousarray(topo.row_ptr, dtype=np.int32),
            np.ascontiguousarray(topo.link_dst, dtype=np.int32),
            np.ascontiguousarray(topo.link_rev, dtype=np.int32),
            np.ascontiguousarray(topo.flow_src, dtype=np.int32),
            np.ascontiguousarray(topo.flow_dst, dtype=np.int32),
            np.ascontiguousarray(topo.flow_rate_bps, dtype=np.uint64)]
    t = _Topo(topo.n_nodes, topo.n_links, topo.n_flows, topo.max_deg, *[a.ctypes.data for a in keep])
    if not topo.identity:                      # identity overlays pass n_overlay = 0
        ov = [np.ascontiguousarray(topo.overlay_nodes, dtype=np.int32),
              np.ascontiguousarray(topo.overlay_adj, dtype=np.int32)]
        keep += ov
        t.n_overlay = topo.n_overlay
        t.overlay_nodes = ov[0].ctypes.data
        t.overlay_adj = ov[1].ctypes.data
    return t, keep


def _params_struct(params: dict) -> _Params:
    """prisma_params_t from an engine_params() dict (engine defaults to auto)."""
    return _Params(**{k: params.get(k, _PARAM_DEFAULTS[k]) if k in _PARAM_DEFAULTS else params[k]
                      for k, _ in _Params._fields_})


def plan(topo: Topology, params: dict) -> dict:
    """prisma_plan: validate a scenario and report its per-replica footprint (no device needed)."""
    L = load_library()
    t, keep = _topo_struct(topo)
    p = _params_struct(params)
    out = _Plan()
    _check(L.prisma_plan(C.byref(t), C.byref(p), C.byref(out)))
    return {k: int(getattr(out, k)) for k, _ in _Plan._fields_}


class PrismaEngine:
    """R replicas of one scenario on one MI355X (device memory owned by the library)."""

    def __init__(self, topo: Topology, params: dict, n_replicas: int, device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise PrismaError("PrismaEngine needs a HIP device (no CPU fallback)")
        L = load_library()
        self.topo = topo
        self.params = dict(params)
        self.R = int(n_replicas)
        self.device = int(device)
        self.torch_device = torch.device("cuda", self.device)
        t, self._keep = _topo_struct(topo)
        p = _params_struct(params)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            _check(L.prisma_create(C.byref(t), C.byref(p), self.R, self.device, C.byref(h)))
        self.h = h
        lv = _LogView()
        _check(L.prisma_log_view(self.h, C.byref(lv)))
        self.W = int(lv.obs_width)
        self.rec_bytes = int(lv.record_bytes)
        self.log_capacity = int(lv.log_capacity)
        self.rec_dtype = record_dtype(self.W)
        sb, lb = C.c_uint32(), C.c_uint32()
        _check(L.prisma_state_bytes(self.h, C.byref(sb), C.byref(lb)))
        self.state_bytes, self.lds_bytes = int(sb.value), int(lb.value)
        # step-kernel instances the library picked (prisma_kernel_info: the choice prisma_create
        # made, reported by the library; the demangled names are for profiles)
        ki = self.kernel_info()
        self.engine_kind = ki["engine"]
        ctrl = "true" if ki["ctrl"] else "false"
        if self.engine_kind == PRISMA_ENGINE_MEMORY:
            self.kernel_name = f"prisma_mem_step_kernel<false, {ctrl}>"
            self.kernel_name_mlp = f"prisma_mem_step_kernel<true, {ctrl}>"
        else:
            fs, ls = ki["flow_slots"], ki["link_slots"]
            tun = "true" if ki["tunnels"] else "false"
            # template arguments: slots, in-kernel MLP, tunnels, --train/notify_dest paths
            self.kernel_name = f"prisma_step_kernel_t<{fs}, {ls}, false, {tun}, {ctrl}>"
            self.kernel_name_mlp = f"prisma_step_kernel_t<{fs}, {ls}, true, {tun}, {ctrl}>"
        self.obs = torch.zeros((self.R, self.W), dtype=torch.int32, device=self.torch_device)
        self.mask = torch.zeros(self.R, dtype=torch.uint8, device=self.torch_device)
        self.node = torch.zeros(self.R, dtype=torch.int32, device=self.torch_device)

    def kernel_info(self) -> dict:
        """prisma_kernel_info: the step-kernel instances this engine launches (engine, template
        slots, tunnels, ctrl paths, relay entries with LDS FIFO windows, relay index bits)."""
        ki = _KernelInfo()
        _check(_lib.prisma_kernel_info(self.h, C.byref(ki)))
        return {k: int(getattr(ki, k)) for k, _ in _KernelInfo._fields_}

    # -- lifecycle --------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            _lib.prisma_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, episode: int = 0, stream=None):
        _check(_lib.prisma_reset(self.h, int(episode), _stream_handle(stream)))

    # -- hot path ---------------------------------------------------------
    def step(self, actions=None, stream=None):
        """Apply actions [R] (int32 on device) to pending decisions, advance to the next ones."""
        a = 0
        if actions is not None:
            if actions.dtype != self.obs.dtype or actions.numel() != self.R or not actions.is_cuda:
                raise PrismaError("actions must be a device int32 tensor of n_replicas elements")
            a = actions.contiguous().data_ptr()
        _check(_lib.prisma_step(self.h, a or None, self.obs.data_ptr(), self.mask.data_ptr(), self.node.data_ptr(),
                                _stream_handle(stream)))
        return self.obs, self.mask, self.node

    def compact_pending(self, stream=None):
        """The pending replicas of the last step() as a dense batch (prisma_compact_pending):
        (ids int32 [n], obs int32 [n, W], node int32 [n]) for a policy that evaluates only the
        notified replicas (ns3env.py:417-423). One host read of the count. The tensors are views
        of buffers the next call reuses: valid until then (clone them to keep them longer)."""
        import torch
        if not hasattr(self, "_cids"):
            self._cids = torch.empty(self.R, dtype=torch.int32, device=self.torch_device)
            self._cobs = torch.empty((self.R, self.W), dtype=torch.int32, device=self.torch_device)
            self._cnode = torch.empty(self.R, dtype=torch.int32, device=self.torch_device)
            self._ccount = torch.zeros(1, dtype=torch.int32, device=self.torch_device)
        _check(_lib.prisma_compact_pending(self.h, self.mask.data_ptr(), self.obs.data_ptr(), self.node.data_ptr(),
                                           self._cids.data_ptr(), self._cobs.data_ptr(), self._cnode.data_ptr(),
                                           self._ccount.data_ptr(), _stream_handle(stream)))
        n = int(self._ccount.item())
        self._cn = n
        return self._cids[:n], self._cobs[:n], self._cnode[:n]

    def expand_actions(self, ids, packed_actions, fill: int = 0, stream=None):
        """Actions of a compacted batch back to one per replica (prisma_expand_actions), ready
        for step(); replicas without a pending decision get `fill`."""
        import torch
        out = torch.empty(self.R, dtype=torch.int32, device=self.torch_device)
        n = int(ids.numel())
        # the count on the device without a host-to-device copy (a pageable copy synchronises the
        # stream): compact_pending's own count when ids is its batch, else a device-side fill
        if (hasattr(self, "_ccount") and n and n == self._cn and ids.data_ptr() == self._cids.data_ptr()
                and ids.dtype == torch.int32):
            cnt = self._ccount
        else:
            # a fresh count per call, filled on the launch's own stream: a reused buffer could be
            # refilled while an earlier expand still reads it, or read before a fill on another stream
            with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream()):
                cnt = torch.full((1,), n, dtype=torch.int32, device=self.torch_device)
        # (an empty batch still passes valid device pointers: the count says there is nothing)
        ids_c = ids.to(torch.int32).contiguous() if n else torch.zeros(1, dtype=torch.int32, device=self.torch_device)
        act = (packed_actions.to(torch.int32).contiguous() if n
               else torch.zeros(1, dtype=torch.int32, device=self.torch_device))
        _check(_lib.prisma_expand_actions(self.h, ids_c.data_ptr(), cnt.data_ptr(), act.data_ptr(), int(fill),
                                          out.data_ptr(), _stream_handle(stream)))
        return out

    def run(self, policy, max_hops: int, stream=None):
        """Fused in-kernel policy: every replica executes up to max_hops hops.

        policy: a device uint8 [N, N] action table (SP, DQ-routing argmin), or the device fp32
        packed DQN-buffer weights of StackedQNet(kind="buffer").pack()."""
        import torch
        n, d = self.topo.n_nodes, self.topo.max_deg
        if not policy.is_cuda:
            raise PrismaError("policy data must live on the device")
        if policy.dtype == torch.uint8 and tuple(policy.shape) == (n, n):
            kind = PRISMA_POLICY_TABLE
        elif policy.dtype == torch.float32 and policy.dim() == 1 and policy.numel() == dqn_buffer_floats(n, d):
            kind = PRISMA_POLICY_DQN_BUFFER
        else:
            raise PrismaError("policy must be a uint8 [n_nodes, n_nodes] table or packed fp32 DQN-buffer weights")
        self._policy_keep = policy.contiguous()
        _check(_lib.prisma_run(self.h, kind, self._policy_keep.data_ptr(), int(max_hops), _stream_handle(stream)))

    # -- outputs ----------------------------------------------------------
    def counters(self, stream=None) -> np.ndarray:
        out = np.zeros(self.R, dtype=COUNTERS_DTYPE)
        _check(_lib.prisma_read_counters(self.h, out.ctypes.data, _stream_handle(stream)))
        return out

    def counters_tensor(self, stream=None):
        """Device copy of the counters as a torch uint8 tensor [R, 144] (for device-side use / collectives)."""
        import torch
        buf = torch.empty((self.R, COUNTERS_DTYPE.itemsize), dtype=torch.uint8, device=self.torch_device)
        _check(_lib.prisma_copy_counters(self.h, buf.data_ptr(), _stream_handle(stream)))
        return buf

    def gather_records(self, replica, dec, stream=None):
        """Device gather of records -> torch uint8 [n, rec_bytes] (replica int32, dec int32/uint32 on device)."""
        import torch
        n = int(replica.numel())
        out = torch.empty((max(n, 1), self.rec_bytes), dtype=torch.uint8, device=self.torch_device)
        if n:
            rep = replica.to(torch.int32).contiguous()
            d = dec.to(torch.int32).contiguous()
            _check(_lib.prisma_gather_records(self.h, rep.data_ptr(), d.data_ptr(), n, out.data_ptr(),
                                              _stream_handle(stream)))
        return out[:n]

    def log_tensor(self, stream=None):
        import torch
        nbytes = self.R * self.log_capacity * self.rec_bytes
        buf = torch.empty(nbytes, dtype=torch.uint8, device=self.torch_device)
        _check(_lib.prisma_copy_log(self.h, buf.data_ptr(), nbytes, _stream_handle(stream)))
        return buf.view(self.R, self.log_capacity, self.rec_bytes)

    def records(self, replica: int, first: int, count: int, log_host: Optional[np.ndarray] = None) -> np.ndarray:
        """Records [first, first+count) of one replica in decision order (host numpy)."""
        if log_host is None:
            import torch
            torch.cuda.synchronize(self.device)
            log_host = self.log_tensor().cpu().numpy()
        if count > self.log_capacity:
            raise PrismaError("requested more records than the log ring holds")
        cap = self.log_capacity
        idx = (np.arange(first, first + count) % cap)
        raw = log_host[replica][idx]
        return raw.reshape(-1).view(self.rec_dtype)
