// mppi_dynamics.cpp -- host rigid-body dynamics of the arm node's robot model (the
// Pinocchio calls of kinova.py:126-184).
//
// The reference node runs, every 10 ms tick, pin.computeAllTerms(model, data, q, v) on
// the free-flyer model of full_robot_floating2.urdf (kinova.py:54-61) and applies the
// computed-torque law
//     tau = M[6:, 6:] @ (400 (qdes - q[7:]) - 40 v[6:]) + nle[6:]        (kinova.py:184)
// to the MPPI output qdes.  Pinocchio is not available here, so this file carries the
// two algorithms that law needs, in double precision, with Pinocchio's conventions:
//   * free-flyer root: q = (xyz, quaternion xyzw), v = (linear, angular) velocity of the
//     base frame expressed in the base frame; revolute / prismatic children;
//   * fixed-joint links merged into their movable ancestor's inertia (as Pinocchio's
//     URDF parser appends fixed bodies);
//   * gravity (0, 0, -g) in the world frame.
// rnea() is Featherstone's recursive Newton-Euler (spatial motion / force vectors as
// (linear, angular) 3-vector pairs at the body origin in body coordinates).  The mass
// matrix is assembled column by column from rnea(q, 0, e_j) without gravity; nle is
// rnea(q, v, 0).  The computed-torque law is ONE rnea pass with a = (0, ades): rows 6..
// of M a + nle, without forming M.
//
// K = 1 per control tick and sequential over the tree: host work, like the reference's
// Pinocchio call (GPU launches would cost more than the whole pass).
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mppi_hip.h"

extern "C" mppi_status mppi_fail_dyn(mppi_status st, const char* msg);   // mppi_host_math.cpp (last_error)

namespace {

struct V3 { double x, y, z; };
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

struct M3 { double m[9]; };
inline V3 mul(const M3& R, V3 v) {
    return {R.m[0] * v.x + R.m[1] * v.y + R.m[2] * v.z, R.m[3] * v.x + R.m[4] * v.y + R.m[5] * v.z,
            R.m[6] * v.x + R.m[7] * v.y + R.m[8] * v.z};
}
inline V3 mulT(const M3& R, V3 v) {   // R^T v
    return {R.m[0] * v.x + R.m[3] * v.y + R.m[6] * v.z, R.m[1] * v.x + R.m[4] * v.y + R.m[7] * v.z,
            R.m[2] * v.x + R.m[5] * v.y + R.m[8] * v.z};
}
inline M3 mul(const M3& A, const M3& B) {
    M3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[3 * i + j] = A.m[3 * i] * B.m[j] + A.m[3 * i + 1] * B.m[3 + j] + A.m[3 * i + 2] * B.m[6 + j];
    return r;
}
inline M3 eye() { return M3{{1, 0, 0, 0, 1, 0, 0, 0, 1}}; }
M3 rpy_matrix(const double* rpy) {   // Rz(y) Ry(p) Rx(r)
    const double cr = std::cos(rpy[0]), sr = std::sin(rpy[0]), cp = std::cos(rpy[1]), sp = std::sin(rpy[1]);
    const double cy = std::cos(rpy[2]), sy = std::sin(rpy[2]);
    return M3{{cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr, sy * cp, sy * sp * sr + cy * cr,
               sy * sp * cr - cy * sr, -sp, cp * sr, cp * cr}};
}
M3 axis_angle(V3 a, double q) {   // Rodrigues about the unit axis a
    const double c = std::cos(q), s = std::sin(q), t = 1.0 - c;
    return M3{{c + a.x * a.x * t, a.x * a.y * t - a.z * s, a.x * a.z * t + a.y * s,
               a.y * a.x * t + a.z * s, c + a.y * a.y * t, a.y * a.z * t - a.x * s,
               a.z * a.x * t - a.y * s, a.z * a.y * t + a.x * s, c + a.z * a.z * t}};
}
M3 quat_xyzw(const double* q) {   // unit quaternion (normalised here, as pin.XYZQUATToSE3)
    const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const double x = q[0] / n, y = q[1] / n, z = q[2] / n, w = q[3] / n;
    return M3{{1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
               2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
               2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)}};
}

struct Body {
    int parent;        // body index, -1 = world
    int type;          // MPPI_JOINT_FLOATING / REVOLUTE / PRISMATIC
    int qi, vi;        // first q / v index of the joint
    M3 Rj;             // joint frame in the parent body frame
    V3 pj;
    V3 axis;           // unit joint axis (joint frame)
    double m;          // merged inertia about the body origin, body frame:
    V3 h;              //   mass, first moment m*c, rotational inertia I_o
    M3 Io;
};

}  // namespace

struct mppi_dyn {
    std::vector<Body> b;
    int nq = 0, nv = 0;
    double g = 9.81;
    std::vector<V3> Vv, Vw, Af, An, Ff, Fn;   // per-body scratch
    std::vector<M3> R;                        // parent -> child rotation of the current pass
    std::vector<V3> p;                        //   and the child origin in the parent frame
};

namespace {

// One recursive Newton-Euler pass: tau = M(q) a + C(q, v) v + g(q) (gravity when grav).
void rnea(mppi_dyn* d, const double* q, const double* v, const double* a, bool grav, double* tau) {
    const int n = (int)d->b.size();
    for (int i = 0; i < n; ++i) {
        const Body& B = d->b[i];
        V3 vv{0, 0, 0}, vw{0, 0, 0}, af{0, 0, 0}, an{0, 0, 0};
        if (B.type == MPPI_JOINT_FLOATING) {   // root: world -> base placement from q
            d->R[i] = quat_xyzw(q + B.qi + 3);
            d->p[i] = {q[B.qi], q[B.qi + 1], q[B.qi + 2]};
            vv = {v[B.vi], v[B.vi + 1], v[B.vi + 2]};
            vw = {v[B.vi + 3], v[B.vi + 4], v[B.vi + 5]};
            if (a) { af = {a[B.vi], a[B.vi + 1], a[B.vi + 2]}; an = {a[B.vi + 3], a[B.vi + 4], a[B.vi + 5]}; }
            if (grav) af = af + mulT(d->R[i], V3{0, 0, d->g});   // -gravity as a base acceleration
        } else {
            const double qj = q[B.qi], vj = v[B.vi], aj = a ? a[B.vi] : 0.0;
            if (B.type == MPPI_JOINT_REVOLUTE) {
                d->R[i] = mul(B.Rj, axis_angle(B.axis, qj));
                d->p[i] = B.pj;
            } else {
                d->R[i] = B.Rj;
                d->p[i] = B.pj + qj * mul(B.Rj, B.axis);
            }
            const M3& Rc = d->R[i];
            const V3 pc = d->p[i];
            V3 pvv{0, 0, 0}, pvw{0, 0, 0}, paf{0, 0, 0}, pan{0, 0, 0};
            if (B.parent >= 0) {
                pvv = d->Vv[B.parent]; pvw = d->Vw[B.parent]; paf = d->Af[B.parent]; pan = d->An[B.parent];
            } else if (grav) {
                paf = V3{0, 0, d->g};
            }
            // motion transform parent -> child: w_c = R^T w_p, v_c = R^T (v_p + w_p x p)
            vw = mulT(Rc, pvw);
            vv = mulT(Rc, pvv + cross(pvw, pc));
            an = mulT(Rc, pan);
            af = mulT(Rc, paf + cross(pan, pc));
            if (B.type == MPPI_JOINT_REVOLUTE) {     // S = (0, axis)
                const V3 s = vj * B.axis;
                // A += S qdd + V x (S qd):  (v x s, w x s)
                af = af + cross(vv, s);
                an = an + aj * B.axis + cross(vw, s);
                vw = vw + s;
            } else {                                 // S = (axis, 0)
                const V3 s = vj * B.axis;
                af = af + aj * B.axis + cross(vw, s);
                vv = vv + s;
            }
        }
        d->Vv[i] = vv; d->Vw[i] = vw; d->Af[i] = af; d->An[i] = an;
        // F = I A + V x* (I V), inertia about the body origin: p = m v + w x h, L = Io w + h x v
        const V3 pl = B.m * vv + cross(vw, B.h);
        const V3 L = mul(B.Io, vw) + cross(B.h, vv);
        const V3 f = B.m * af + cross(an, B.h);
        const V3 nn = mul(B.Io, an) + cross(B.h, af);
        d->Ff[i] = f + cross(vw, pl);
        d->Fn[i] = nn + cross(vw, L) + cross(vv, pl);
    }
    for (int i = n - 1; i >= 0; --i) {
        const Body& B = d->b[i];
        const V3 f = d->Ff[i], nn = d->Fn[i];
        if (B.type == MPPI_JOINT_FLOATING) {
            tau[B.vi] = f.x; tau[B.vi + 1] = f.y; tau[B.vi + 2] = f.z;
            tau[B.vi + 3] = nn.x; tau[B.vi + 4] = nn.y; tau[B.vi + 5] = nn.z;
        } else {
            tau[B.vi] = (B.type == MPPI_JOINT_REVOLUTE) ? dot(B.axis, nn) : dot(B.axis, f);
        }
        if (B.parent >= 0) {   // force transform child -> parent: f_p = R f, n_p = R n + p x f_p
            const V3 fp = mul(d->R[i], f);
            d->Ff[B.parent] = d->Ff[B.parent] + fp;
            d->Fn[B.parent] = d->Fn[B.parent] + mul(d->R[i], nn) + cross(d->p[i], fp);
        }
    }
}

}  // namespace

extern "C" {

mppi_status mppi_dyn_create(const mppi_link* links, int32_t n, double gravity, mppi_dyn** out) {
    if (!links || n < 1 || n > 256 || !out) return mppi_fail_dyn(MPPI_ERR_INVALID_ARG, "mppi_dyn_create: bad arguments");
    *out = nullptr;
    auto* d = new mppi_dyn();
    d->g = gravity;
    std::vector<int> body_of(n, -1);
    std::vector<M3> Rin(n);      // link frame in its body frame
    std::vector<V3> pin_(n);
    for (int i = 0; i < n; ++i) {
        const mppi_link& L = links[i];
        if (L.parent >= i || L.parent < -1 || L.type < 0 || L.type > 3) {
            delete d;
            return mppi_fail_dyn(MPPI_ERR_INVALID_ARG, "mppi_dyn_create: links must be topologically ordered with valid types");
        }
        if (L.type == MPPI_JOINT_FLOATING && L.parent != -1) {
            delete d;
            return mppi_fail_dyn(MPPI_ERR_INVALID_ARG, "mppi_dyn_create: a floating joint must attach to the world");
        }
        const M3 Ro = rpy_matrix(L.rpy);
        const V3 po{L.xyz[0], L.xyz[1], L.xyz[2]};
        if (L.type == MPPI_JOINT_FIXED) {
            if (L.parent < 0) { delete d; return mppi_fail_dyn(MPPI_ERR_INVALID_ARG, "mppi_dyn_create: fixed link under the world"); }
            body_of[i] = body_of[L.parent];
            Rin[i] = mul(Rin[L.parent], Ro);
            pin_[i] = pin_[L.parent] + mul(Rin[L.parent], po);
        } else {
            Body B{};
            B.parent = (L.parent >= 0) ? body_of[L.parent] : -1;
            B.type = L.type;
            if (L.type == MPPI_JOINT_FLOATING) {
                B.qi = d->nq; B.vi = d->nv; d->nq += 7; d->nv += 6;
                B.Rj = eye(); B.pj = {0, 0, 0};
            } else {
                B.qi = d->nq; B.vi = d->nv; d->nq += 1; d->nv += 1;
                const M3& Rp = (L.parent >= 0) ? Rin[L.parent] : eye();
                const V3 pp = (L.parent >= 0) ? pin_[L.parent] : V3{0, 0, 0};
                B.Rj = mul(Rp, Ro);
                B.pj = pp + mul(Rp, po);
            }
            V3 ax{L.axis[0], L.axis[1], L.axis[2]};
            const double an = std::sqrt(dot(ax, ax));
            B.axis = (an > 0) ? (1.0 / an) * ax : V3{1, 0, 0};
            B.m = 0.0; B.h = {0, 0, 0};
            std::memset(B.Io.m, 0, sizeof(B.Io.m));
            body_of[i] = (int)d->b.size();
            Rin[i] = eye();
            pin_[i] = {0, 0, 0};
            d->b.push_back(B);
        }
        // accumulate the link's inertial into its body: COM c and inertia about the COM Ic
        // (link frame) -> body frame, then about the body origin (parallel axis)
        Body& B = d->b[body_of[i]];
        const double m = L.mass;
        const V3 c = pin_[i] + mul(Rin[i], V3{L.com[0], L.com[1], L.com[2]});
        M3 Ic;
        std::memcpy(Ic.m, L.inertia, sizeof(Ic.m));
        M3 RIc = mul(mul(Rin[i], Ic), M3{{Rin[i].m[0], Rin[i].m[3], Rin[i].m[6], Rin[i].m[1], Rin[i].m[4],
                                           Rin[i].m[7], Rin[i].m[2], Rin[i].m[5], Rin[i].m[8]}});
        const double cc = dot(c, c);
        const double cv[3] = {c.x, c.y, c.z};
        for (int r = 0; r < 3; ++r)
            for (int s = 0; s < 3; ++s) B.Io.m[3 * r + s] += RIc.m[3 * r + s] + m * ((r == s ? cc : 0.0) - cv[r] * cv[s]);
        B.m += m;
        B.h = B.h + m * c;
    }
    const size_t nb = d->b.size();
    d->Vv.resize(nb); d->Vw.resize(nb); d->Af.resize(nb); d->An.resize(nb); d->Ff.resize(nb); d->Fn.resize(nb);
    d->R.resize(nb); d->p.resize(nb);
    *out = d;
    return MPPI_OK;
}

void mppi_dyn_destroy(mppi_dyn* d) { delete d; }

void mppi_dyn_dims(const mppi_dyn* d, int32_t* nq, int32_t* nv, int32_t* nbodies) {
    if (nq) *nq = d ? d->nq : 0;
    if (nv) *nv = d ? d->nv : 0;
    if (nbodies) *nbodies = d ? (int32_t)d->b.size() : 0;
}

mppi_status mppi_dyn_rnea(mppi_dyn* d, const double* q, const double* v, const double* a, double* tau) {
    if (!d || !q || !v || !tau) return mppi_fail_dyn(MPPI_ERR_INVALID_ARG, "mppi_dyn_rnea: bad arguments");
    rnea(d, q, v, a, true, tau);
    return MPPI_OK;
}

mppi_status mppi_dyn_terms(mppi_dyn* d, const double* q, const double* v, double* M, double* nle) {
    if (!d || !q || !v || (!M && !nle)) return mppi_fail_dyn(MPPI_ERR_INVALID_ARG, "mppi_dyn_terms: bad arguments");
    const int nv = d->nv;
    if (nle) rnea(d, q, v, nullptr, true, nle);
    if (M) {
        std::vector<double> zero(nv, 0.0), e(nv, 0.0), col(nv);
        for (int j = 0; j < nv; ++j) {
            e[j] = 1.0;
            rnea(d, q, zero.data(), e.data(), false, col.data());
            e[j] = 0.0;
            for (int i = 0; i < nv; ++i) M[i * nv + j] = col[i];
        }
        for (int i = 0; i < nv; ++i)   // symmetrise (the two triangles agree to rounding)
            for (int j = i + 1; j < nv; ++j) {
                const double s = 0.5 * (M[i * nv + j] + M[j * nv + i]);
                M[i * nv + j] = s; M[j * nv + i] = s;
            }
    }
    return MPPI_OK;
}

mppi_status mppi_computed_torque(mppi_dyn* d, const double* q, const double* v, const double* qdes, double kp,
                                 double kd, int32_t first_v, double* tau) {
    if (!d || !q || !v || !qdes || !tau || first_v < 0 || first_v > d->nv)
        return mppi_fail_dyn(MPPI_ERR_INVALID_ARG, "mppi_computed_torque: bad arguments");
    const int nv = d->nv, nact = nv - first_v;
    const int first_q = d->nq - nact;   // the actuated joints are the trailing 1-dof joints
    std::vector<double> a(nv, 0.0), t(nv);
    for (int j = 0; j < nact; ++j)   // ades = kp (qdes - q) - kd v   (kinova.py:184)
        a[first_v + j] = kp * (qdes[j] - q[first_q + j]) + kd * (-v[first_v + j]);
    rnea(d, q, v, a.data(), true, t.data());   // = (M a + nle) rows first_v..
    for (int j = 0; j < nact; ++j) tau[j] = t[first_v + j];
    return MPPI_OK;
}

}  // extern "C"
