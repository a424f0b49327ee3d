"""Active-replica compaction (prisma_compact_pending / prisma_expand_actions, include/prisma.h
ABI 9): a batched external policy evaluates only the replicas with a pending decision, as the
reference's Forwarder steps only the notified nodes (/root/reference/prisma/ns3_model/ns3env.py:
417-423). Checked against torch's masked selection and against the uncompacted step sequence."""
import numpy as np
import pytest
import torch

from prisma_amd.config import engine_params
from prisma_amd.engine import PRISMA_ENGINE_MEMORY, PrismaEngine
from prisma_amd.topology import Topology, sp_next_hop_table

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not torch.cuda.is_available(), reason="needs an MI355X")]


def _actions(obs, node, table):
    """SP table actions for rows (obs[:, 0] = destination), 0 for rows without a node."""
    nd = node.long().clamp_min(0)
    return torch.where(node >= 0, table[nd, obs[:, 0].long().clamp(0, table.shape[1] - 1)].int(),
                       torch.zeros_like(node))


@pytest.mark.parametrize("name,R,engine", [("abilene", 4096, 0), ("abilene", 1000, 0), ("geant", 777, PRISMA_ENGINE_MEMORY)])
def test_compacted_policy_equals_full_policy(name, R, engine):
    """Two engines stepped in lock-step: one with the policy on every row, one through the
    compacted batch. The compacted rows equal torch's masked selection (ascending ids), and the
    two engines' observations, masks and logs stay identical, across 0.4-s episode ends with
    auto-reset. Prints the measured active fraction."""
    topo = Topology.example(name, 0, 2.0)
    params = engine_params(topo, sim_time_s=0.4, ping_as_obs=0, notify_dest=1, auto_reset=1, engine=engine)
    table = torch.from_numpy(sp_next_hop_table(topo)).cuda()
    a, b = PrismaEngine(topo, params, R), PrismaEngine(topo, params, R)
    a.reset(0)
    b.reset(0)
    oa, ma, na = a.step(None)
    ob, mb, nb = b.step(None)
    active, steps, empty_seen = 0, 0, 0
    for s in range(2000):
        ids, obs_p, node_p = b.compact_pending()
        sel = torch.nonzero(mb.bool()).squeeze(1).int()
        assert torch.equal(ids, sel), s
        assert torch.equal(obs_p, ob[sel.long()]) and torch.equal(node_p, nb[sel.long()]), s
        active += int(ids.numel())
        steps += 1
        empty_seen += int(ids.numel() < R)
        act_b = b.expand_actions(ids, _actions(obs_p, node_p, table), fill=0)
        act_a = _actions(oa, na, table)
        act_a = torch.where(ma.bool(), act_a, torch.zeros_like(act_a))
        assert torch.equal(act_a, act_b), s
        oa, ma, na = a.step(act_a)
        ob, mb, nb = b.step(act_b)
        assert torch.equal(oa, ob) and torch.equal(ma, mb) and torch.equal(na, nb), s
    torch.cuda.synchronize()
    ca, cb = a.counters(), b.counters()
    assert ca.tobytes() == cb.tobytes()
    assert int(ca["episode"].min()) >= 1                   # the run crossed episode ends
    frac = active / (steps * R)
    print(f"\n[compact] {name} R={R}: active fraction {frac:.5f} over {steps} steps "
          f"({empty_seen} steps with an inactive replica)")
    assert 0.0 < frac <= 1.0
    a.close()
    b.close()


def test_compaction_of_sparse_and_empty_masks():
    """Masks of every density, including none and all, at ragged sizes."""
    topo = Topology.example("abilene")
    for R in (1, 63, 64, 65, 1023, 1024, 1025, 5000):
        eng = PrismaEngine(topo, engine_params(topo), R)
        g = torch.Generator(device="cuda").manual_seed(R)
        for p in (0.0, 0.01, 0.5, 1.0):
            eng.mask.copy_((torch.rand(R, device="cuda", generator=g) < p).to(torch.uint8))
            eng.obs.copy_(torch.randint(0, 1 << 20, eng.obs.shape, device="cuda", generator=g, dtype=torch.int32))
            eng.node.copy_(torch.randint(-1, 11, (R,), device="cuda", generator=g, dtype=torch.int32))
            ids, obs_p, node_p = eng.compact_pending()
            sel = torch.nonzero(eng.mask.bool()).squeeze(1)
            assert torch.equal(ids.long(), sel) and torch.equal(obs_p, eng.obs[sel]) and torch.equal(node_p, eng.node[sel])
            packed = torch.arange(ids.numel(), device="cuda", dtype=torch.int32) + 7
            full = eng.expand_actions(ids, packed, fill=-3)
            want = torch.full((R,), -3, dtype=torch.int32, device="cuda")
            want[sel] = packed
            assert torch.equal(full, want)
        eng.close()
