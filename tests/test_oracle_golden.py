"""Pin the CPU oracle against golden vectors produced by the reference's own code
(tests/golden/make_golden.py)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import egnn_mc, graph, gravity, ponita, rollout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fc_edge_index_matches_reference(golden):
    g = golden("graph")
    n = 0
    for k in g.files:
        if k.startswith("fc_"):
            B, N = map(int, k.split("_")[1:])
            np.testing.assert_array_equal(graph.fc_edge_index(B, N), g[k])
            n += 1
    assert n == 5


def test_knn_edge_index_matches_reference(golden):
    g = golden("graph")
    for k in g.files:
        if k.startswith("knn_") and not k.endswith("_loc"):
            B, N, kk = map(int, k.split("_")[1:])
            np.testing.assert_array_equal(graph.build_graph_with_knn(g[k + "_loc"], B, N, kk), g[k])


def test_knn_k_ge_n_raises(golden):
    assert int(golden("graph")["k_ge_n_raises"]) == 1
    with pytest.raises(ValueError):
        graph.build_graph_with_knn(np.zeros((5, 3)), 1, 5, 5)


def test_gravity_acceleration_matches_reference(golden):
    gv = golden("gravity")
    np.testing.assert_array_equal(gravity.compute_acceleration(gv["acc_pos"], gv["acc_mass"], 2.0, 0.2), gv["acc_out"])


@pytest.mark.parametrize("N,T,seed", [(5, 1000, 0), (5, 1000, 1), (5, 1000, 2), (5, 1000, 3), (100, 100, 0),
                                      (100, 100, 1)])
def test_gravity_trajectory_matches_reference(golden, N, T, seed):
    gv = golden("gravity")
    p, v, m = gravity.initial_conditions(N, seed)
    ps, vs, fs = gravity.sample_trajectories(p[None], v[None], m[None], T=T, sample_freq=10, dt=0.01, G=2.0,
                                             softening=0.2)
    pre = f"traj_N{N}_T{T}_s{seed}_"
    np.testing.assert_array_equal(ps[0], gv[pre + "pos"])
    np.testing.assert_array_equal(vs[0], gv[pre + "vel"])
    np.testing.assert_array_equal(fs[0], gv[pre + "force"])
    np.testing.assert_array_equal(m, gv[pre + "mass"])


@pytest.fixture(scope="module")
def c_oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "liboracle_gravity.so"))
    lib.oracle_gravity_sample.restype = ctypes.c_int
    return lib


def run_c_oracle(lib, pos, vel, mass, T, freq, dt=0.01, G=2.0, soft=0.2):
    S, N, _ = pos.shape
    pos, vel = np.ascontiguousarray(pos, np.float64).copy(), np.ascontiguousarray(vel, np.float64).copy()
    mass = np.ascontiguousarray(mass.reshape(S, N), np.float64)
    Ts = T // freq
    outs = [np.zeros((S, Ts, N, 3)) for _ in range(3)]
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = lib.oracle_gravity_sample(ctypes.c_int64(S), ctypes.c_int64(N), ctypes.c_int64(T), ctypes.c_int64(freq),
                                   ctypes.c_double(dt), ctypes.c_double(G), ctypes.c_double(soft), P(pos), P(vel),
                                   P(mass), *[P(o) for o in outs])
    assert rc == 0
    return outs


def test_c_oracle_matches_reference(golden, c_oracle):
    gv = golden("gravity")
    p, v, m = gravity.initial_conditions(5, 0)
    ps, vs, fs = run_c_oracle(c_oracle, p[None], v[None], m[None], 1000, 10)
    pre = "traj_N5_T1000_s0_"
    # C pow/summation order differs from numpy/BLAS in the last ulp; 5-body chaos
    # amplifies it over 1000 steps, so compare the first 20 frames tightly.
    np.testing.assert_allclose(ps[0, :20], gv[pre + "pos"][:20], rtol=0, atol=1e-10)
    np.testing.assert_allclose(vs[0, :20], gv[pre + "vel"][:20], rtol=0, atol=1e-10)
    np.testing.assert_allclose(fs[0, :20], gv[pre + "force"][:20], rtol=0, atol=1e-9)


def _params(npz, tag):
    pre = f"{tag}/param/"
    return {k[len(pre):]: npz[k].astype(np.float64) for k in npz.files if k.startswith(pre)}


@pytest.mark.parametrize("tag,tol", [("f64", 1e-13), ("f32", 1e-6)])
def test_ponita_oracle_matches_reference(golden, tag, tol):
    P = golden("ponita")
    p = _params(P, tag)
    grid = P[f"{tag}/ori_grid"].astype(np.float64)
    loc, vel, mass = P["loc"].reshape(-1, 3), P["vel"].reshape(-1, 3), P["mass"].reshape(-1, 1)
    ei = graph.fc_edge_index(4, 5)
    out = ponita.forward(p, mass, vel[:, None, :], ei, loc[ei[0]] - loc[ei[1]], grid, 2)
    np.testing.assert_allclose(out, P[f"{tag}/pred"], rtol=0, atol=tol)
    L, V = rollout.rollout(rollout.ponita_step(p, grid, 2), P["loc"], P["vel"], P["force"], P["mass"], 10)
    np.testing.assert_allclose(L, P[f"{tag}/roll_loc"], rtol=0, atol=50 * tol)
    np.testing.assert_allclose(V, P[f"{tag}/roll_vel"], rtol=0, atol=50 * tol)


@pytest.mark.parametrize("tag,tol", [("f64", 1e-13), ("f32", 1e-6)])
def test_egnn_mc_oracle_matches_reference(golden, tag, tol):
    E = golden("egnn_mc")
    p = _params(E, tag)
    loc, vel, mass = E["loc"].reshape(-1, 3), E["vel"].reshape(-1, 3), E["mass"].reshape(-1, 1)
    ei = graph.fc_edge_index(4, 5)
    x, ea = egnn_mc.preprocess(loc, vel, mass, ei)
    np.testing.assert_allclose(egnn_mc.forward(p, x, loc, vel, ei, ea, 2), E[f"{tag}/pred"], rtol=0, atol=tol)
    L, V = rollout.rollout(rollout.egnn_mc_step(p, 2), E["loc"], E["vel"], E["force"], E["mass"], 10)
    np.testing.assert_allclose(L, E[f"{tag}/roll_loc"], rtol=0, atol=50 * tol)
    np.testing.assert_allclose(V, E[f"{tag}/roll_vel"], rtol=0, atol=50 * tol)
