"""Routing agents restated in PyTorch (the reference's are TF 2.8 / networkx).

* ``SPPolicy`` — forwarder.py:190-191: ``neighbors.index(nx.shortest_path(G,
  u, dst)[1])``, as a [N, N] next-hop table (topology.sp_next_hop_table, pinned
  against networkx fixtures).
* ``StackedQNet(kind="routing")`` — models.py:360-392 DQN_routing_model:
  one_hot(dst, N) -> Dense(32) -> Dense(64) -> Dense(64) -> Dense(deg), ELU
  on every layer, he_uniform kernels AND biases (Keras fan_in of a bias =
  its length).
* ``StackedQNet(kind="buffer")`` — models.py:258-306 DQN_buffer_model: the
  one-hot branch Dense(32) || LayerNormalization(axis=1, no centre/scale,
  epsilon 1e-3 = Keras default) of the deg buffer values -> Dense(32); concat
  -> Dense(64) -> Dense(64) -> Dense(deg), ELU everywhere.
* action = argmin_a Q(obs)[a] (learner.py:142-145), first index on ties,
  greedy (train=0, forwarder.py:183-186).

One network per overlay node (the reference's per-node agents), stored
stacked over UNDERLAY node ids (rows of non-overlay nodes stay zero; the one-hot
input is obs[0], the destination's overlay index, so W1 rows past N_o are
unused), with the action/input dimension padded to max_deg so a
whole batch of decisions at different nodes is ONE set of batched GEMMs
(torch.bmm over the gathered per-node weights), not a Python loop over nodes.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from .topology import Topology, sp_next_hop_table


class SPPolicy:
    """obs[0] is the destination's overlay index (data-packet-manager.cc:175); the table
    is indexed by underlay ids (node, destination)."""

    def __init__(self, topo: Topology, device="cuda"):
        self.topo = topo
        self.table = torch.from_numpy(sp_next_hop_table(topo)).to(device)
        self.dst_of = torch.from_numpy(topo.overlay_nodes.astype(np.int64)).to(device)

    def act(self, obs: torch.Tensor, node: torch.Tensor) -> torch.Tensor:
        dst = self.dst_of[obs[:, 0].long().clamp(0, self.dst_of.numel() - 1)]
        return self.table[node.long(), dst].to(torch.int32)


def _he_uniform(gen: torch.Generator, fan_in: int, shape) -> torch.Tensor:
    lim = math.sqrt(6.0 / fan_in)
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2.0 - 1.0).mul_(lim).to(torch.float32)


class StackedQNet(torch.nn.Module):
    """Per-node Q networks of one topology, stacked on a leading node axis."""

    def __init__(self, topo: Topology, kind: str = "routing", seed: int = 0, device="cuda"):
        super().__init__()
        if kind not in ("routing", "buffer"):
            raise ValueError("kind must be 'routing' or 'buffer'")
        self.kind = kind
        self.N = topo.n_nodes
        self.topo_overlay_nodes = topo.overlay_nodes.astype(np.int64)
        self.D = topo.max_deg
        deg = torch.from_numpy(topo.degrees.astype(np.int64))
        self.register_buffer("deg", deg)
        g = torch.Generator().manual_seed(int(seed))
        N, D = self.N, self.D

        def dense(fan_ins, din_pad, dout, dout_pad=None):
            dout_pad = dout if dout_pad is None else dout_pad
            W = torch.zeros(N, din_pad, dout_pad)
            b = torch.zeros(N, dout_pad)
            for u in range(N):
                fi = int(fan_ins[u])
                do = int(dout[u]) if not isinstance(dout, int) else dout
                if int(topo.degrees[u]) == 0:
                    continue                                  # not an overlay node: no agent
                W[u, :fi, :do] = _he_uniform(g, fi, (fi, do))
                b[u, :do] = _he_uniform(g, do, (do,))
            return torch.nn.Parameter(W), torch.nn.Parameter(b)

        ones = [topo.n_overlay] * N                                 # one_hot(dst, numNodes)
        self.W1, self.b1 = dense(ones, N, 32)                       # one-hot(dst) branch
        if kind == "buffer":
            self.Wb, self.bb = dense(topo.degrees, D, 32)           # buffers branch (deg inputs)
            self.W2, self.b2 = dense([64] * N, 64, 64)
        else:
            self.W2, self.b2 = dense([32] * N, 32, 64)
        self.W3, self.b3 = dense([64] * N, 64, 64)
        self.W4, self.b4 = dense([64] * N, 64, [int(d) for d in topo.degrees], D)
        self.to(device)

    @staticmethod
    def _lin(x, W, b, node):
        return torch.bmm(x.unsqueeze(1), W[node]).squeeze(1) + b[node]

    def q_values(self, obs: torch.Tensor, node: torch.Tensor) -> torch.Tensor:
        """Q [B, max_deg] for observations obs [B, >=1+deg] at nodes node [B]; padded actions = +inf."""
        node = node.long()
        dst = obs[:, 0].long()
        elu = torch.nn.functional.elu
        h1 = elu(self.W1[node, dst] + self.b1[node])                # one_hot @ W1 == row gather
        if self.kind == "buffer":
            D = self.D
            deg = self.deg[node]
            x = obs[:, 1:1 + D].to(torch.float32)
            valid = (torch.arange(D, device=x.device)[None, :] < deg[:, None])
            cnt = deg.to(torch.float32)[:, None]
            xm = torch.where(valid, x, torch.zeros_like(x))
            mean = xm.sum(1, keepdim=True) / cnt
            var = (torch.where(valid, x - mean, torch.zeros_like(x)) ** 2).sum(1, keepdim=True) / cnt
            xn = torch.where(valid, (x - mean) / torch.sqrt(var + 1e-3), torch.zeros_like(x))
            hb = elu(self._lin(xn, self.Wb, self.bb, node))
            h = torch.cat([h1, hb], dim=1)
        else:
            h = h1
        h = elu(self._lin(h, self.W2, self.b2, node))
        h = elu(self._lin(h, self.W3, self.b3, node))
        q = elu(self._lin(h, self.W4, self.b4, node))
        pad = torch.arange(self.D, device=q.device)[None, :] >= self.deg[node][:, None]
        return q.masked_fill(pad, float("inf"))

    @torch.no_grad()
    def act(self, obs: torch.Tensor, node: torch.Tensor) -> torch.Tensor:
        return torch.argmin(self.q_values(obs, node), dim=1).to(torch.int32)

    @torch.no_grad()
    def pack(self) -> torch.Tensor:
        """Flat fp32 weights for the in-kernel DQN-buffer policy (PRISMA_POLICY_DQN_BUFFER):
        W1[N][N][32] b1[N][32] Wb[N][D][32] bb[N][32] W2[N][64][64] b2[N][64] W3[N][64][64]
        b3[N][64] W4[N][64][D] b4[N][D] (include/prisma.h)."""
        if self.kind != "buffer":
            raise ValueError("pack() is the DQN-buffer layout (kind='buffer')")
        parts = [self.W1, self.b1, self.Wb, self.bb, self.W2, self.b2, self.W3, self.b3, self.W4, self.b4]
        return torch.cat([p.detach().to(torch.float32).contiguous().flatten() for p in parts])

    @torch.no_grad()
    def argmin_table(self) -> torch.Tensor:
        """[N, N] uint8 action table by underlay ids (node, destination); valid for
        kind='routing' (Q depends on (node, dst) only).  Rows / columns of non-overlay
        nodes are 0."""
        if self.kind != "routing":
            raise ValueError("only the DQ-routing model has a state-independent argmin table")
        dev = self.W1.device
        # the (node, destination) grid is built once per device: a host-to-device copy per call
        # (from pageable memory, non_blocking=False) synchronises the stream, so every policy
        # refresh would wait for the engine launch before it and leave the GPU idle meanwhile
        key = str(dev)
        if getattr(self, "_grid_dev", None) != key:
            on = torch.from_numpy(self.topo_overlay_nodes).to(dev)
            no = on.numel()
            obs = torch.zeros((no * no, 1 + self.D), dtype=torch.int32, device=dev)
            obs[:, 0] = torch.arange(no, device=dev).repeat(no).to(torch.int32)
            self._grid = (on, on.repeat_interleave(no), obs)
            self._grid_dev = key
        on, node, obs = self._grid
        no = on.numel()
        a = self.act(obs, node).view(no, no)
        a.fill_diagonal_(0)                                   # at destination: action 0 (forwarder.py:149)
        table = torch.zeros((self.N, self.N), dtype=torch.uint8, device=dev)
        table[on[:, None], on[None, :]] = a.to(torch.uint8)
        return table
