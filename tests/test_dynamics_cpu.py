"""Host rigid-body dynamics of the arm node (kinova.py:126-184)
against the independent numpy Lagrangian in ``oracle/dynamics_oracle.py``.  PARITY
UNPINNED with respect to the reference's Pinocchio (not installed, no committed
outputs).  Pure CPU: the C++ code in libmppi_hip.so runs on the host."""
import numpy as np
import pytest

from oracle.dynamics_oracle import TreeModel
from quadrotor_manipulator_mppi_amd.robot.dynamics import RobotDynamics
from quadrotor_manipulator_mppi_amd.robot.urdf_tree import load_tree

HOME = [1.57, 1.7, 0.0, 4.4, 0.0, 4.71, 0.0]    # kinova.py:135


def _states(n=4, seed=0):
    rng = np.random.default_rng(seed)
    out = [(np.array([0, 0, 1.0, 0, 0, 0, 1.0] + HOME), np.zeros(13))]
    for _ in range(n):
        quat = rng.normal(size=4)
        quat /= np.linalg.norm(quat)
        q = np.concatenate([rng.uniform(-1, 1, 3), quat, np.array(HOME) + rng.uniform(-1, 1, 7)])
        out.append((q, rng.normal(0, 1.0, 13)))
    return out


@pytest.fixture(scope="module")
def models():
    tree = load_tree()
    return RobotDynamics(tree), TreeModel(tree)


def test_model_shape(models):
    d, o = models
    assert (d.nq, d.nv, d.n_bodies) == (14, 13, 8)   # free-flyer + 7 revolute; fixed links merged
    M, nle = d.compute_all_terms(*_states()[0])
    assert abs(M[0, 0] - sum(l["mass"] for l in load_tree())) < 1e-12


def test_mass_matrix_matches_lagrangian(models):
    d, o = models
    for q, v in _states():
        M, _ = d.compute_all_terms(q, v)
        Mo = o.mass_matrix(q)
        assert np.allclose(M, Mo, rtol=1e-10, atol=1e-12), np.abs(M - Mo).max()
        assert np.allclose(M, M.T) and np.linalg.eigvalsh(M).min() > 0


def test_gravity_matches_lagrangian(models):
    d, o = models
    for q, _ in _states():
        _, g = d.compute_all_terms(q, np.zeros(13))
        assert np.allclose(g, o.gravity(q), rtol=1e-10, atol=1e-10)


def test_joint_nle_matches_lagrangian(models):
    """Coriolis + centrifugal + gravity on the joint rows (the rows kinova.py:184 uses)."""
    d, o = models
    for q, v in _states():
        _, nle = d.compute_all_terms(q, v)
        ref = o.nle_joint_rows(q, v)
        assert np.allclose(nle[6:], ref, rtol=1e-5, atol=1e-6), np.abs(nle[6:] - ref).max()


def test_power_balance_all_rows(models):
    """v^T C(q,v) v = 1/2 v^T Mdot v over all 13 rows (base rows included)."""
    d, o = models
    for q, v in _states()[1:]:
        _, nle = d.compute_all_terms(q, v)
        _, g = d.compute_all_terms(q, np.zeros(13))
        lhs = v @ (nle - g)
        rhs = 0.5 * v @ o.mdot(q, v) @ v
        assert abs(lhs - rhs) <= 1e-5 * max(1.0, abs(rhs))


def test_rnea_is_M_a_plus_nle(models):
    d, _ = models
    rng = np.random.default_rng(3)
    for q, v in _states():
        a = rng.normal(size=13)
        M, nle = d.compute_all_terms(q, v)
        assert np.allclose(d.rnea(q, v, a), M @ a + nle, rtol=1e-11, atol=1e-9)


def test_computed_torque_is_kinova_184(models):
    """tau = M[6:,6:] (400 (qdes - q[7:]) - 40 v[6:]) + nle[6:] (kinova.py:184)."""
    d, _ = models
    rng = np.random.default_rng(4)
    for q, v in _states():
        qdes = q[7:] + rng.normal(0, 0.01, 7)
        M, nle = d.compute_all_terms(q, v)
        want = M[6:, 6:] @ (400 * (qdes - q[7:]) + 40 * (-v[6:])) + nle[6:]
        assert np.allclose(d.computed_torque(q, v, qdes), want, rtol=1e-11, atol=1e-9)


def test_fixed_base_arm_variant():
    """A fixed-base tree (the arm alone, its base placement folded into joint 1's origin)
    through the same C++: its M equals the free-flyer model's joint block M[6:,6:] (which
    does not depend on the base), and its gravity equals nle[6:] at v = 0 with the
    free-flyer base at identity."""
    from scipy.spatial.transform import Rotation
    tree = load_tree()
    arm = [dict(l) for l in tree[2:]]                      # link_1 .. fingers
    base_joint, j1 = tree[1], tree[2]
    Rb = Rotation.from_euler("xyz", base_joint["rpy"]).as_matrix()   # URDF rpy = Rz Ry Rx
    R1 = Rotation.from_euler("xyz", j1["rpy"]).as_matrix()
    arm[0]["rpy"] = list(Rotation.from_matrix(Rb @ R1).as_euler("xyz"))
    arm[0]["xyz"] = list(Rb @ np.asarray(j1["xyz"]) + np.asarray(base_joint["xyz"]))
    arm[0]["parent"] = -1
    for l in arm[1:]:
        l["parent"] -= 2
    fixed = RobotDynamics(arm)
    assert (fixed.nq, fixed.nv) == (7, 7)
    flo = RobotDynamics(tree)
    rng = np.random.default_rng(5)
    for _ in range(4):
        qa = np.array(HOME) + rng.uniform(-1, 1, 7)
        quat = rng.normal(size=4)
        quat /= np.linalg.norm(quat)
        Mf, _ = flo.compute_all_terms(np.concatenate([[0.3, -0.2, 1.0], quat, qa]), rng.normal(size=13))
        Ma, ga = fixed.compute_all_terms(qa, np.zeros(7))
        assert np.allclose(Ma, Mf[6:, 6:], rtol=1e-11, atol=1e-12)
        _, g0 = flo.compute_all_terms(np.concatenate([[0, 0, 0], [0, 0, 0, 1.0], qa]), np.zeros(13))
        assert np.allclose(ga, g0[6:], rtol=1e-10, atol=1e-10)
