"""GPU parity: HIP graph builder and GravitySim integrator vs the oracle / golden
vectors.  Edge indices must be bit-exact; the fp64 integrator is compared per
step (ulp-level) and over short horizons (5-body chaos amplifies last-bit
differences of pow/summation order over long runs)."""
import numpy as np
import pytest
import torch

from oracle import graph as og
from oracle import gravity as ogr

pytestmark = pytest.mark.gpu


def test_fc_edge_index_bit_exact(hip_device, golden):
    import nbody_amd.graph as G
    g = golden("graph")
    for k in g.files:
        if k.startswith("fc_"):
            B, N = map(int, k.split("_")[1:])
            np.testing.assert_array_equal(G.fc_edge_index(B, N, hip_device).cpu().numpy(), g[k])
    for B, N in [(1024, 5), (4096, 5), (3, 100), (7, 1), (0, 5)]:
        ei = G.build_graph_with_knn(None, B, N, hip_device, None).cpu().numpy()
        np.testing.assert_array_equal(ei, og.fc_edge_index(B, N).reshape(2, -1))


def test_knn_edge_index(hip_device, golden):
    import nbody_amd.graph as G
    g = golden("graph")
    for k in g.files:
        if k.startswith("knn_") and not k.endswith("_loc"):
            B, N, kk = map(int, k.split("_")[1:])
            loc = torch.tensor(g[k + "_loc"], device=hip_device)
            np.testing.assert_array_equal(G.build_graph_with_knn(loc, B, N, hip_device, kk).cpu().numpy(), g[k])
    with pytest.raises(ValueError):
        G.build_graph_with_knn(torch.zeros(5, 3, device=hip_device), 1, 5, hip_device, 5)


def test_gravity_acceleration(hip_device, golden):
    from nbody_amd.gravity import GravitySim
    gv = golden("gravity")
    acc = GravitySim.compute_acceleration(gv["acc_pos"], gv["acc_mass"], 2.0, 0.2)
    np.testing.assert_allclose(acc, gv["acc_out"], rtol=1e-14, atol=1e-14)


@pytest.mark.parametrize("N,T,seed", [(5, 1000, 0), (5, 1000, 3), (100, 100, 1)])
def test_gravity_trajectory_vs_reference(hip_device, golden, N, T, seed):
    from nbody_amd.gravity import GravitySim
    gv = golden("gravity")
    sim = GravitySim(n_balls=N, interaction_strength=2, dt=0.01, softening=0.2, device=hip_device)
    p, v, f, m = sim.sample_trajectory(T=T, sample_freq=10, random_seed=seed)
    pre = f"traj_N{N}_T{T}_s{seed}_"
    k = 20 if T >= 200 else T // 10
    np.testing.assert_allclose(p[:k], gv[pre + "pos"][:k], rtol=0, atol=1e-9)
    np.testing.assert_allclose(v[:k], gv[pre + "vel"][:k], rtol=0, atol=1e-9)
    np.testing.assert_allclose(f[:k], gv[pre + "force"][:k], rtol=0, atol=1e-8)
    assert np.array_equal(p[0], gv[pre + "pos"][0])        # frame 0 = initial state, bit-exact


def test_gravity_batched_energy_property(hip_device):
    """Full-batch property: the KDK integrator is symplectic, so total energy of
    every system stays close to its initial value — same drift as the oracle."""
    from nbody_amd.gravity import GravitySim
    S, N, T = 256, 5, 1000
    sim = GravitySim(n_balls=N, interaction_strength=2, dt=0.01, softening=0.2, device=hip_device)
    ics = [sim.initial_conditions(s) for s in range(S)]
    pos = np.stack([c[0] for c in ics]); vel = np.stack([c[1] for c in ics]); mass = np.stack([c[2] for c in ics])
    ps, vs, _ = sim.sample_trajectories(pos, vel, mass, T=T, sample_freq=10)
    ps, vs = ps.cpu().numpy(), vs.cpu().numpy()
    e0 = np.array([ogr.energy(ps[s, 0], vs[s, 0], mass[s], 2.0, 0.2)[2] for s in range(S)])
    e1 = np.array([ogr.energy(ps[s, -1], vs[s, -1], mass[s], 2.0, 0.2)[2] for s in range(S)])
    rel = np.abs(e1 - e0) / np.abs(e0)
    assert np.median(rel) < 1e-2
    # first 5 frames of every system match the numpy oracle to ulp-level growth
    rp, rv, _ = ogr.sample_trajectories(pos, vel, mass, T=50, sample_freq=10, dt=0.01, G=2.0, softening=0.2)
    np.testing.assert_allclose(ps[:, :5], rp, rtol=0, atol=1e-11)


def test_gravity_multi_system_n100_every_workgroup_slot(hip_device):
    """C5's shape (N = 100: 10 systems per 1,000-lane workgroup, gravity.hip): 23 systems fill two
    workgroups and leave a partial third (3 of 10 slots), so every local slot 0-9 and the partial
    last workgroup are exercised.  Each system must match the numpy oracle (bit-exact with the
    reference per DESIGN §2; synthetic_sim.py:357-420) over 10 frames, and equal the same system
    integrated alone (slot 0 of a one-system launch) bit for bit."""
    from nbody_amd.gravity import GravitySim
    S, N, T, f = 23, 100, 100, 10
    sim = GravitySim(n_balls=N, interaction_strength=2, dt=0.01, softening=0.2, device=hip_device)
    ics = [sim.initial_conditions(100 + s) for s in range(S)]
    pos = np.stack([c[0] for c in ics]); vel = np.stack([c[1] for c in ics]); mass = np.stack([c[2] for c in ics])
    ps, vs, fs = (t.cpu().numpy() for t in sim.sample_trajectories(pos, vel, mass, T=T, sample_freq=f))
    assert ps.shape == (S, T // f, N, 3)
    rp, rv, rf = ogr.sample_trajectories(pos, vel, mass, T=T, sample_freq=f, dt=0.01, G=2.0, softening=0.2)
    np.testing.assert_array_equal(ps[:, 0], pos)              # frame 0 = the initial state, bit-exact
    np.testing.assert_allclose(ps, rp, rtol=0, atol=1e-9)
    np.testing.assert_allclose(vs, rv, rtol=0, atol=1e-9)
    np.testing.assert_allclose(fs, rf, rtol=0, atol=1e-8)
    np.testing.assert_allclose(ps[:, :5], rp[:, :5], rtol=0, atol=1e-11)
    for s in range(S):
        one = [t.cpu().numpy()[0] for t in sim.sample_trajectories(pos[s:s + 1], vel[s:s + 1], mass[s:s + 1],
                                                                      T=T, sample_freq=f)]
        for a, b in zip((ps[s], vs[s], fs[s]), one):
            np.testing.assert_array_equal(a, b)
