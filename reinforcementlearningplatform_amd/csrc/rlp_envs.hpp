// rlp_envs.hpp — batched environment dynamics, one env per lane, float64 physics in registers.
//
// Each Env<KIND> restates one reference env copy's step_update / get_state / reset
// (citations per function, relative to the reference root). Expression order follows the
// reference (numpy evaluates left to right and never fuses multiply-adds; the library is built
// with -ffp-contract=off), float32-action quirks under NumPy-2 promotion included, so results match
// the reference numpy step() to ~1 ulp of libm rather than to the 1e-5 the contract allows.
#pragma once
#include "rlp_common.hpp"

namespace rlp {

constexpr double kPi = 3.141592653589793;
__device__ __forceinline__ double deg2rad(double d) { return d * kPi / 180.; }
__device__ __forceinline__ double clipd(double x, double lo, double hi) {
    return x < lo ? lo : (x > hi ? hi : x);
}

// fp64 sin and cos of one argument: Cody-Waite reduction by pi/2 (three-part constant, FMA) and
// the classic minimax kernels on [-pi/4, pi/4] (fdlibm __kernel_sin/__kernel_cos coefficients),
// <= 1 ulp like libm for |x| < 2^20 (accuracy degrades beyond: no live episode gets there, every
// env terminates at |angle| of a few rad). ~30 VALU ops instead of the general-purpose routine's
// ~150 plus its call — the physics' sub-step loops call it 4x per sub-step.
__device__ __forceinline__ void sincos_fast(double x, double *sp, double *cp) {
    const double kd = rint(x * 0.63661977236758134308);
    double r = fma(-kd, 1.5707963267948966192, x);
    r = fma(-kd, 6.123233995736766036e-17, r);
    r = fma(-kd, -1.4973849048591698e-33, r);
    const double z = r * r;
    // sin(r) = r + r^3 (S1 + z (S2 + ... z S6))
    const double ps = fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                        2.75573137070700676789e-06), -1.98412698298579493134e-04),
                          8.33333333332248946124e-03);
    const double sr = r + (z * r) * fma(z, ps, -1.66666666666666324348e-01);
    // cos(r) = w + ((1 - w) - z/2 + z^2 (C1 + z (C2 + ... z C6))), w = 1 - z/2
    const double pc = z * fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11,
                                                           2.08757232129817482790e-09),
                                                    -2.75573143513906633035e-07),
                                             2.48015872894767294178e-05),
                                      -1.38888888888741095749e-03),
                               4.16666666666666019037e-02);
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * pc);
    const int q = ((int)kd) & 3;
    const double s0 = (q & 1) ? cr : sr, c0 = (q & 1) ? sr : cr;
    *sp = (q & 2) ? -s0 : s0;
    *cp = ((q + 1) & 2) ? -c0 : c0;
}

// sin / cos of theta + d for an RK4 stage offset d (h * dtheta / 2 or h * dtheta) from sb, cb =
// sin / cos theta: the angle-addition identities with d's sine and cos - 1 from their Taylor
// series to d^11 / d^12 (truncation < 2e-19 for |d| <= 0.25, i.e. |dtheta| < 125 rad/s at CartPole's
// h = 2 ms, and < 2e-14 at |d| = 0.5), the small corrections added last: within ~1 ulp of
// sincos_fast(theta + d) at ~19 VALU ops instead of ~35.
__device__ __forceinline__ void sincos_step(double sb, double cb, double d, double *sp, double *cp) {
    const double z = d * d;
    // sin d = d + d z (-1/3! + z (1/5! + z (-1/7! + z (1/9! - z / 11!))))
    const double ps = fma(z, fma(z, fma(z, fma(z, -2.505210838544172e-08, 2.755731922398589e-06),
                                        -1.984126984126984e-04), 8.333333333333333e-03),
                          -1.666666666666667e-01);
    const double sd = fma(d * z, ps, d);
    // cos d - 1 = z (-1/2! + z (1/4! + z (-1/6! + z (1/8! + z (-1/10! + z / 12!)))))
    const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, 2.087675698786810e-09, -2.755731922398589e-07),
                                                  2.48015873015873e-05), -1.388888888888889e-03),
                                 4.166666666666667e-02), -0.5);
    const double cm1 = z * pc;
    *sp = sb + fma(sb, cm1, cb * sd);
    *cp = cb + fma(cb, cm1, -(sb * sd));
}

// x / 6 (the RK4 average): x * (1/6) plus one FMA residual correction (Markstein) — the correctly
// rounded quotient but for rare ties, <= 1 ulp always; 3 VALU ops instead of the ~12 of the
// general f64 division (scale / rcp / Newton / fmas / fixup)
__device__ __forceinline__ double div6(double x) {
    constexpr double r6 = 1.0 / 6.0;
    const double q = x * r6;
    return fma(fma(-6.0, q, x), r6, q);
}

// num / den for a finite, normal den (every physics denominator here: masses, inertias,
// M + m - 3/4 m cos^2, cos(theta) away from 0): v_rcp_f64 + two Newton steps + a residual
// correction, <= 1 ulp (no scaling / special-value path: 8 VALU ops instead of ~12)
__device__ __forceinline__ double div_nr(double num, double den) {
    double y = __builtin_amdgcn_rcp(den);
    y = fma(y, fma(-den, y, 1.0), y);
    y = fma(y, fma(-den, y, 1.0), y);
    const double q = num * y;
    return fma(fma(-den, q, num), y, q);
}

// Reciprocal of a finite, normal den (rcp + two Newton steps, <= 1 ulp) and the quotient from it
// with one residual correction (Markstein): for denominators shared by several quotients in a step
// (inertias, mass, cos theta), 3 VALU ops per quotient after the reciprocal's 5.
__device__ __forceinline__ double recip_nr(double den) {
    double y = __builtin_amdgcn_rcp(den);
    y = fma(y, fma(-den, y, 1.0), y);
    return fma(y, fma(-den, y, 1.0), y);
}
__device__ __forceinline__ double div_r(double num, double den, double y) {
    const double q = num * y;
    return fma(fma(-den, q, num), y, q);
}

// exp / log / tanh for the UAV controller and reward (FNTSMC.py:96-106, UavHoverOuterLoop.py:93-110):
// ~20-40 VALU ops each instead of ocml's 42 / 98 / 165 (whose double-double paths buy the last
// half ulp): <= 2-3 ulp, far inside the 1e-9 state parity (tests/test_gpu_rollout_parity.py).
// exp: Cody-Waite by ln 2 (hi / lo), Taylor to r^13 on |r| <= ln2/2 (truncation < 1e-17), ldexp;
// the argument clamped to [-746, 709.7] (exp(-inf) = 0, as pow(0, a > 0) = 0).
__device__ __forceinline__ double exp_fast(double x) {
    x = fmin(fmax(x, -746.0), 709.78);
    const double k = rint(x * 1.4426950408889634074);
    double r = fma(-k, 6.93147180369123816490e-01, x);
    r = fma(-k, 1.90821492927058770002e-10, r);
    double q = 1.6059043836821614599e-10;                 // 1/13!
    q = fma(q, r, 2.0876756987868098979e-09);             // 1/12!
    q = fma(q, r, 2.5052108385441718775e-08);             // 1/11!
    q = fma(q, r, 2.7557319223985890653e-07);             // 1/10!
    q = fma(q, r, 2.7557319223985890653e-06);             // 1/9!
    q = fma(q, r, 2.4801587301587301587e-05);             // 1/8!
    q = fma(q, r, 1.9841269841269841270e-04);             // 1/7!
    q = fma(q, r, 1.3888888888888888889e-03);             // 1/6!
    q = fma(q, r, 8.3333333333333333333e-03);             // 1/5!
    q = fma(q, r, 4.1666666666666666667e-02);             // 1/4!
    q = fma(q, r, 1.6666666666666666667e-01);             // 1/3!
    q = fma(q, r, 0.5);
    q = fma(q, r, 1.0);
    q = fma(q, r, 1.0);
    return __builtin_amdgcn_ldexp(q, (int)k);
}
// log: x = m 2^e with m in [sqrt(1/2), sqrt(2)), f = m - 1 exact, s = f / (2 + f), and fdlibm's
// __ieee754_log reduction and minimax coefficients Lg1..Lg7 (< 1 ulp there); log(0) = -inf.
__device__ __forceinline__ double log_fast(double x) {
    double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
    int e = __builtin_amdgcn_frexp_exp(x);
    const bool lo = m < 0.70710678118654752440;
    m = lo ? m + m : m;
    e = lo ? e - 1 : e;
    const double f = m - 1.0, dk = (double)e;
    const double s = div_nr(f, 2.0 + f);
    const double z = s * s, w = z * z;
    const double t1 = w * fma(w, fma(w, 1.531383769920937332e-01, 2.222219843214978396e-01),
                              3.999999999940941908e-01);
    const double t2 = z * fma(w, fma(w, fma(w, 1.479819860511658591e-01, 1.818357216161805012e-01),
                                     2.857142874366239149e-01), 6.666666666666735130e-01);
    const double R = t2 + t1, hfsq = 0.5 * f * f;
    const double r = dk * 6.93147180369123816490e-01 -
                     ((hfsq - (s * (hfsq + R) + dk * 1.90821492927058770002e-10)) - f);
    return x == 0.0 ? -__builtin_inf() : r;
}
// tanh(x) = sign(x) em / (em + 2), em = expm1(2|x|) = 2^k (1 + q) - 1 with q = expm1(r) (Taylor to
// r^14 on |r| <= ln2/2): relative accuracy for tiny |x| (k = 0: em = q), |x| clamped to 22
// (tanh = 1 in f64 beyond 19.1).
__device__ __forceinline__ double tanh_fast(double x) {
    const double y = 2.0 * fmin(fabs(x), 22.0);
    const double k = rint(y * 1.4426950408889634074);
    double r = fma(-k, 6.93147180369123816490e-01, y);
    r = fma(-k, 1.90821492927058770002e-10, r);
    double q = 1.1470745597729724714e-11;                 // 1/14!
    q = fma(q, r, 1.6059043836821614599e-10);
    q = fma(q, r, 2.0876756987868098979e-09);
    q = fma(q, r, 2.5052108385441718775e-08);
    q = fma(q, r, 2.7557319223985890653e-07);
    q = fma(q, r, 2.7557319223985890653e-06);
    q = fma(q, r, 2.4801587301587301587e-05);
    q = fma(q, r, 1.9841269841269841270e-04);
    q = fma(q, r, 1.3888888888888888889e-03);
    q = fma(q, r, 8.3333333333333333333e-03);
    q = fma(q, r, 4.1666666666666666667e-02);
    q = fma(q, r, 1.6666666666666666667e-01);
    q = fma(q, r, 0.5);
    q = r * fma(q, r, 1.0);                               // expm1(r)
    const int ki = (int)k;
    const double em = __builtin_amdgcn_ldexp(q, ki) + (__builtin_amdgcn_ldexp(1.0, ki) - 1.0);
    return copysign(div_nr(em, em + 2.0), x);
}

// The same object behind an opaque (scalar) pointer: loads of its fields after this point cannot
// reuse values loaded before it, so a long step re-reads its parameters phase by phase (short
// SGPR live ranges) instead of holding them all at once — the UAV step's ~60 uniform doubles
// otherwise spill to VGPR lanes (a v_readlane per use). Only for objects in memory (the rollout
// kernel's kernarg segment), never a by-value copy.
template <class T>
__device__ __forceinline__ const T &phase_ref(const T &x) {
    const T *q = &x;
    asm volatile("" : "+s"(q));
    return *q;
}

template <int KIND> struct Env;

// components of the physics state step() may change (E::DW when the kind declares it, else D):
// the step kernel writes back only those
template <class E, class = void> struct EnvDW { static constexpr int value = E::D; };
template <class E> struct EnvDW<E, std::void_t<decltype(E::DW)>> { static constexpr int value = E::DW; };

// ==========================================================================================
// CartPole — environment/CartPole/CartPole.py (PPO2 and DPPO2 demo copies via params)
// state: theta, dtheta, x, dx, time
// ==========================================================================================
template <> struct Env<RLP_ENV_CARTPOLE> {
    using P = rlp_cartpole_params;
    static constexpr int D = RLP_CARTPOLE_D, S = 4, A = 1;

    // CartPole.ode :219-238 (sin / cos of xx[0] given), the products and sums contracted into FMAs
    // (15 -> 10 f64 ops besides the division; each differs from numpy's two roundings by <= 1 ulp,
    // like the fast sincos and the Newton division: parity to the reference is 1e-9, not bits)
    __device__ static __forceinline__ void ode_sc(const P &p, double force, const double xx[4],
                                                  double Sv, double Cv, double d[4]) {
        const double dth = xx[1], dx = xx[3];
        const double mell = p.m * p.ell, c1 = 3.0 / 4.0 * p.m * p.g, c2 = 3.0 / 4.0 * p.m;
        const double c3 = 3.0 / 4.0 / p.m / p.ell, mg = p.m * p.g, Mm = p.M + p.m;  // uniform
        double num = fma(mell * dth * dth, Sv, force);
        num = fma(-p.kf, dx, num);
        num = fma(-(c1 * Sv), Cv, num);
        const double den = fma(-(c2 * Cv), Cv, Mm);
        const double ddx = div_nr(num, den);
        const double ddth = c3 * fma(-(p.m * ddx), Cv, mg * Sv);
        d[0] = dth; d[1] = ddth; d[2] = dx; d[3] = ddx;
    }
    __device__ static __forceinline__ void ode(const P &p, double force, const double xx[4],
                                               double d[4]) {
        double Sv, Cv;
        sincos_fast(xx[0], &Sv, &Cv);
        ode_sc(p, force, xx, Sv, Cv, d);
    }
    // get_state :145-153
    __device__ static __forceinline__ void observe(const P &p, const double *s, float *o) {
        o[0] = (float)((s[0] / p.theta_max) * p.static_gain);
        o[1] = (float)((s[1] / p.dtheta_max) * p.static_gain);
        o[2] = (float)((s[2] / p.x_max) * p.static_gain);
        o[3] = (float)((s[3] / p.dx_max) * p.static_gain);
    }
    // step_update :257-264 -> rk44 :240-255, is_Terminal :160-185, get_reward :187-217
    __device__ static __forceinline__ void step(const P &p, double *s, const float *a, float *on,
                                                double &reward, int &flag, bool &done) {
        const float af = a[0];
        const double force = (double)af;
        const double h = p.dt / (double)p.n_sub_div;
        double time = s[4];
        const double tt = time + p.dt;
        double xx[4] = {s[0], s[1], s[2], s[3]};
        while (time < tt) {  // fp64 time accumulation => 10 or 11 sub-steps
            // (K1 + 2*K2 + 2*K3 + K4) / 6 evaluates left to right: a running sum is bit-identical.
            // xx + K/2 and sum + 2K as one FMA each: the power-of-two products are exact, so the
            // single rounding equals numpy's. Stage angles theta + K/2 etc. take sin / cos from the
            // sub-step's sincos by angle addition (sincos_step of the stage offset tmp - theta).
            double sum[4], tmp[4], d[4], S0, C0, Ss, Cs;
            sincos_fast(xx[0], &S0, &C0);
            ode_sc(p, force, xx, S0, C0, d);
#pragma unroll
            for (int i = 0; i < 4; ++i) { const double k = h * d[i]; sum[i] = k; tmp[i] = fma(k, 0.5, xx[i]); }
            sincos_step(S0, C0, tmp[0] - xx[0], &Ss, &Cs);
            ode_sc(p, force, tmp, Ss, Cs, d);
#pragma unroll
            for (int i = 0; i < 4; ++i) { const double k = h * d[i]; sum[i] = fma(k, 2.0, sum[i]); tmp[i] = fma(k, 0.5, xx[i]); }
            sincos_step(S0, C0, tmp[0] - xx[0], &Ss, &Cs);
            ode_sc(p, force, tmp, Ss, Cs, d);
#pragma unroll
            for (int i = 0; i < 4; ++i) { const double k = h * d[i]; sum[i] = fma(k, 2.0, sum[i]); tmp[i] = xx[i] + k; }
            sincos_step(S0, C0, tmp[0] - xx[0], &Ss, &Cs);
            ode_sc(p, force, tmp, Ss, Cs, d);
#pragma unroll
            for (int i = 0; i < 4; ++i) xx[i] = xx[i] + div6(sum[i] + h * d[i]);
            time += h;
        }
        s[0] = xx[0]; s[1] = xx[1]; s[2] = xx[2]; s[3] = xx[3]; s[4] = time;
        const double th = xx[0], dth = xx[1], x = xx[2], dx = xx[3];
        const double eth = 0. - th, ex = 0. - x;
        int f = 0;
        if ((th > p.theta_max + deg2rad(1)) || th < -p.dtheta_max - deg2rad(1)) f = 1;  // :167 (sic)
        if (x > p.x_max || x < -p.x_max) f = 2;
        if (time > p.time_max) f = 3;
        if (sqrt(ex * ex + dx * dx + eth * eth + dth * dth) < 1e-2) f = 4;
        observe(p, s, on);
        const double r_x = -fabs(x) * p.Q_x;
        const double r_dx = -fabs(dx) * p.Q_dx;
        const double r_th = -fabs(th) * p.Q_theta;
        const double r_om = -fabs(dth) * p.Q_omega;
        const double r_f = (double)(-fabsf(af) * (float)p.R);  // float32 (np.float32 force)
        double r_extra = 0.;
        if (f == 1 || f == 2) {
            const double n_ = (p.time_max - time) / p.dt;
            r_extra = n_ * (r_x + r_dx + r_th + r_om + r_f);
        }
        reward = r_x + r_dx + r_th + r_om + r_f + r_extra;
        flag = f;
        done = f != 0;
    }
    // reset(random=True) :272-282
    __device__ static __forceinline__ void reset(const P &p, double *s, uint64_t seed,
                                                 uint64_t counter, uint64_t env_id) {
        double u[2];
        philox_u01_f64x2(seed, counter, env_id, 0x200u, u);
        s[0] = p.reset_theta_lo + (p.reset_theta_hi - p.reset_theta_lo) * u[0];
        s[1] = 0.;
        s[2] = p.reset_x_lo + (p.reset_x_hi - p.reset_x_lo) * u[1];
        s[3] = 0.;
        s[4] = 0.;
    }
};

// ==========================================================================================
// CartPoleAngleOnly — demonstration/PPO2/PPO2-4-CartPoleAngleOnly/cartpole_angleonly.py (variant
// 0, == the DPPO2 copy) and environment/CartPole/CartPoleAngleOnly.py (variant 1), include/rlp.h
// ==========================================================================================
template <> struct Env<RLP_ENV_CARTPOLE_ANGLEONLY> {
    using P = rlp_angleonly_params;
    static constexpr int D = RLP_ANGLEONLY_D, S = 2, A = 1;

    __device__ static __forceinline__ void ode(const P &p, double force, const double xx[4],
                                               double d[4]) {  // :197-216
        double th = xx[0], dth = xx[1], dx = xx[3];
        double Sv, Cv;
        sincos_fast(th, &Sv, &Cv);
        double num = force + p.m * p.ell * (dth * dth) * Sv;
        num = num - p.kf * dx;
        num = num - 3.0 / 4.0 * p.m * p.g * Sv * Cv;
        double den = p.M + p.m - 3.0 / 4.0 * p.m * (Cv * Cv);
        double ddx = div_nr(num, den);
        double ddth = 3.0 / 4.0 / p.m / p.ell * (p.m * p.g * Sv - p.m * ddx * Cv);
        d[0] = dth; d[1] = ddth; d[2] = dx; d[3] = ddx;
    }
    __device__ static __forceinline__ void observe(const P &p, const double *s, float *o) {
        o[0] = (float)((s[0] / p.theta_max) * p.static_gain);  // :137-143
        o[1] = (float)((s[1] / p.norm_dtheta) * p.static_gain);
    }
    // one classic RK4 step of h (running-sum average, bit-identical, see CartPole)
    __device__ static __forceinline__ void rk4(const P &p, double force, double h, double xx[4]) {
        double sum[4], tmp[4], d[4];
        ode(p, force, xx, d);
#pragma unroll
        for (int i = 0; i < 4; ++i) { const double k = h * d[i]; sum[i] = k; tmp[i] = fma(k, 0.5, xx[i]); }
        ode(p, force, tmp, d);
#pragma unroll
        for (int i = 0; i < 4; ++i) { const double k = h * d[i]; sum[i] = fma(k, 2.0, sum[i]); tmp[i] = fma(k, 0.5, xx[i]); }
        ode(p, force, tmp, d);
#pragma unroll
        for (int i = 0; i < 4; ++i) { const double k = h * d[i]; sum[i] = fma(k, 2.0, sum[i]); tmp[i] = xx[i] + k; }
        ode(p, force, tmp, d);
#pragma unroll
        for (int i = 0; i < 4; ++i) xx[i] = xx[i] + div6(sum[i] + h * d[i]);
    }
    __device__ static __forceinline__ double abs_deg(const P &p, double th) {
        // |rad2deg(state[0] / staticGain * thetaMax)| of the obs array (env file :187-188)
        const double o = th / p.theta_max * p.static_gain;
        return fabs(o / p.static_gain * p.theta_max * 180. / kPi);
    }
    __device__ static __forceinline__ void step(const P &p, double *s, const float *a, float *on,
                                                double &reward, int &flag, bool &done) {
        const float af = a[0];
        const double force = (double)af, dt = p.dt;
        const double th0 = s[0];
        double xx[4] = {s[0], s[1], s[2], s[3]};
        double time = s[4];
        if (p.variant == RLP_ANGLEONLY_ENV_FILE) {   // rk44 :231-244: fp64 `while time < tt`
            const double h = dt / (double)p.n_sub_div, tt = time + dt;
            while (time < tt) {
                rk4(p, force, h, xx);
                time += h;
            }
        } else {                                      // rk44 :218-229: one step of dt
            rk4(p, force, dt, xx);
            time = time + dt;
        }
        s[0] = xx[0]; s[1] = xx[1]; s[2] = xx[2]; s[3] = xx[3]; s[4] = time;
        const double th = xx[0], dth = xx[1], eth = 0. - th;
        const bool out = (th > p.theta_max + deg2rad(1)) || th < -p.theta_max - deg2rad(1);
        observe(p, s, on);
        int f = 0;
        if (p.variant == RLP_ANGLEONLY_ENV_FILE) {
            f = out ? 1 : (time > p.time_max ? 3 : 0);     // is_Terminal :144-166 (returns early)
            const double cur = abs_deg(p, th0), nex = abs_deg(p, th);   // get_reward :168-208
            double r = nex > cur ? -2. : (nex == cur ? 0. : 2.);
            if (cur <= 0.5 && nex <= 0.5) r += 5.;
            if (f == 1) r -= 100.;
            else if (f == 3) r += 500.;
            reward = r;
        } else {
            if (out) f = 1;  // is_Terminal :150-168 (later checks override)
            if (time > p.time_max) f = 3;
            if (sqrt(eth * eth + dth * dth) < 1e-2) f = 4;
            const double r1 = -(th * th) * p.Q_theta;  // get_reward :170-195
            const double r2 = -(dth * dth) * p.Q_omega;
            const double r3 = (double)(-(af * af) * (float)p.R);
            double r4 = 0.;
            if (f == 1) {
                const double n_ = (p.time_max - time) / p.dt;
                r4 = n_ * (r1 + r2 + r3);
            }
            reward = r1 + r2 + r3 + r4;
        }
        flag = f;
        done = f != 0;
    }
    __device__ static __forceinline__ void reset(const P &p, double *s, uint64_t seed,
                                                 uint64_t counter, uint64_t env_id) {
        double u[2];  // reset :245-279
        philox_u01_f64x2(seed, counter, env_id, 0x200u, u);
        s[0] = p.reset_theta_lo + (p.reset_theta_hi - p.reset_theta_lo) * u[0];
        s[1] = 0.; s[2] = 0.; s[3] = 0.; s[4] = 0.;
    }
};

// ==========================================================================================
// SecondOrderIntegration — environment/SecondOrderIntegration/SecondOrderIntegration.py
// state: x, y, vx, vy, time, tx, ty
// ==========================================================================================
template <> struct Env<RLP_ENV_SOI> {
    using P = rlp_soi_params;
    static constexpr int D = RLP_SOI_D, S = 4, A = 2;
    static constexpr int DW = 5;  // step() changes x y vx vy time (the target is fixed per episode)

    __device__ static __forceinline__ void observe(const P &p, const double *s, float *o) {
        const double ex = s[5] - s[0], ey = s[6] - s[1];  // get_state :211-219
        o[0] = (float)((ex / p.map_size[0]) * p.obs_gain);
        o[1] = (float)((ey / p.map_size[1]) * p.obs_gain);
        o[2] = (float)((-s[2] / p.v_max) * p.obs_gain);
        o[3] = (float)((-s[3] / p.v_max) * p.obs_gain);
    }
    __device__ static __forceinline__ void step(const P &p, double *s, const float *a, float *on,
                                                double &reward, int &flag, bool &done) {
        const double f0 = (double)a[0], f1 = (double)a[1];
        const double h = p.dt / 1;
        double time = s[4];
        const double tt = time + p.dt;
        while (time < tt) {  // rk44 :298-314 (the loop runs once)
            const double x0 = s[0], x1 = s[1], x2 = s[2], x3 = s[3];
            double K1[4], K2[4], K3[4], K4[4];
            K1[0] = h * x2; K1[1] = h * x3; K1[2] = h * (f0 - p.k * x2); K1[3] = h * (f1 - p.k * x3);
            double t2 = x2 + K1[2] / 2, t3 = x3 + K1[3] / 2;
            K2[0] = h * t2; K2[1] = h * t3; K2[2] = h * (f0 - p.k * t2); K2[3] = h * (f1 - p.k * t3);
            t2 = x2 + K2[2] / 2; t3 = x3 + K2[3] / 2;
            K3[0] = h * t2; K3[1] = h * t3; K3[2] = h * (f0 - p.k * t2); K3[3] = h * (f1 - p.k * t3);
            t2 = x2 + K3[2]; t3 = x3 + K3[3];
            K4[0] = h * t2; K4[1] = h * t3; K4[2] = h * (f0 - p.k * t2); K4[3] = h * (f1 - p.k * t3);
            s[0] = x0 + div6(K1[0] + 2 * K2[0] + 2 * K3[0] + K4[0]);
            s[1] = x1 + div6(K1[1] + 2 * K2[1] + 2 * K3[1] + K4[1]);
            s[2] = x2 + div6(K1[2] + 2 * K2[2] + 2 * K3[2] + K4[2]);
            s[3] = x3 + div6(K1[3] + 2 * K2[3] + 2 * K3[3] + K4[3]);
            time += h;
        }
        s[4] = time;
        const double accx = (f0 - p.k * s[2]) / p.mass, accy = (f1 - p.k * s[3]) / p.mass;
        const double ex = s[5] - s[0], ey = s[6] - s[1];
        const double adm = p.admissible_error;
        int f = 0;  // is_Terminal :235-249
        if (s[0] > p.map_size[0] + adm || s[0] < 0 - adm || s[1] > p.map_size[1] + adm ||
            s[1] < 0 - adm)
            f = 1;
        if (time > p.time_max) f = 2;
        const double e_pos = sqrt(ex * ex + ey * ey), e_vel = sqrt(s[2] * s[2] + s[3] * s[3]);
        if (p.success_enabled && e_pos <= 0.05 && e_vel < 0.05) f = 3;
        observe(p, s, on);
        const double acc = sqrt(accx * accx + accy * accy);  // get_reward :251-284
        const double u_pos = -e_pos * p.Q_pos, u_vel = -e_vel * p.Q_vel, u_acc = -acc * p.Q_acc;
        double u_extra = 0.;
        if (f == 1) {
            const double n_ = (p.time_max - time) / p.dt;
            u_extra = n_ * (u_pos + u_vel + u_acc);
        }
        reward = u_pos + u_vel + u_acc + u_extra;
        flag = f;
        done = f != 0;
    }
    __device__ static __forceinline__ void reset(const P &p, double *s, uint64_t seed,
                                                 uint64_t counter, uint64_t env_id) {
        double u[2];  // reset :328-352
        philox_u01_f64x2(seed, counter, env_id, 0x200u, u);
        const double lo = 0 + p.reset_margin;
        s[0] = lo + ((p.map_size[0] - p.reset_margin) - lo) * u[0];
        s[1] = lo + ((p.map_size[1] - p.reset_margin) - lo) * u[1];
        s[2] = 0.; s[3] = 0.; s[4] = 0.;
        s[5] = p.map_size[0] / 2; s[6] = p.map_size[1] / 2;
    }
};

// ==========================================================================================
// UGVForward / UGVBidirectional — environment/UGV/UGVForward.py, UGVBidirectional.py
// state: x, y, vel, phi, omega, time, tx, ty
// ==========================================================================================
template <bool BIDIR> struct UGV {
    using P = rlp_ugv_params;
    static constexpr int D = RLP_UGV_D, S = 4, A = 2;
    static constexpr int DW = 6;  // step() changes x y vel phi omega time (not the target)

    __device__ static __forceinline__ double get_e(const double *s, double c, double sn) {
        const double ex = s[6] - s[0], ey = s[7] - s[1];
        const double v = sqrt(ex * ex + ey * ey);
        if (!BIDIR) return v;  // UGVForward.get_e :315-317
        const double dot = c * ex + sn * ey;  // UGVBidirectional.get_e
        return (dot > 0 ? 1.0 : (dot < 0 ? -1.0 : 0.0)) * v;
    }
    // get_e_phi -> utils/functions.py:49-60 cal_vector_rad_oriented (+ Bidirectional fold)
    __device__ static __forceinline__ double get_e_phi(const double *s, double c, double sn) {
        const double x2 = s[6] - s[0], y2 = s[7] - s[1];
        double ph;
        if (sqrt(x2 * x2 + y2 * y2) < 1e-4 || sqrt(c * c + sn * sn) < 1e-4) {
            ph = 0;
        } else {
            const double dot = c * x2 + sn * y2;
            const double det = c * y2 - sn * x2;
            ph = atan2(det, dot);
        }
        if (BIDIR) {
            ph = ph >= kPi / 2 ? ph - kPi : ph;
            ph = ph <= -kPi / 2 ? ph + kPi : ph;
        }
        return ph;
    }
    __device__ static __forceinline__ void obs_from(const P &p, const double *s, double e,
                                                    double eph, float *o) {  // get_state :217-227
        const double e_max = sqrt(p.map_size[0] * p.map_size[0] + p.map_size[1] * p.map_size[1]) / 2;
        double s0, s1;
        if (!BIDIR) {
            s0 = 2 / e_max * e - 1;
            s1 = 2 / p.v_max * s[2] - 1;
        } else {
            s0 = e / e_max;
            s1 = s[2] / p.v_max;
        }
        o[0] = (float)(s0 * p.static_gain);
        o[1] = (float)(s1 * p.static_gain);
        o[2] = (float)((eph / kPi) * p.static_gain);
        o[3] = (float)((s[4] / p.omega_max) * p.static_gain);
    }
    __device__ static __forceinline__ void observe(const P &p, const double *s, float *o) {
        double sn, c;
        sincos_fast(s[3], &sn, &c);
        obs_from(p, s, get_e(s, c, sn), get_e_phi(s, c, sn), o);
    }
    __device__ static __forceinline__ void ode(const P &p, double al, double aa, const double *x,
                                               double *d) {  // ode :281-292
        double sn, c;
        sincos_fast(x[3], &sn, &c);
        d[0] = x[2] * c;
        d[1] = x[2] * sn;
        d[2] = al - p.kf * x[2];
        d[3] = x[4];
        d[4] = aa - p.kt * x[4];
    }
    __device__ static __forceinline__ void step(const P &p, double *s, const float *a, float *on,
                                                double &reward, int &flag, bool &done) {
        const double al = (double)a[0], aa = (double)a[1], dt = p.dt;
        double xx[5] = {s[0], s[1], s[2], s[3], s[4]};
        double sum[5], t[5], d[5];  // running RK4 sum (bit-identical, see CartPole)
        ode(p, al, aa, xx, d);  // rk44 :294-313
#pragma unroll
        for (int i = 0; i < 5; ++i) { const double k = dt * d[i]; sum[i] = k; t[i] = fma(k, 0.5, xx[i]); }
        ode(p, al, aa, t, d);
#pragma unroll
        for (int i = 0; i < 5; ++i) { const double k = dt * d[i]; sum[i] = fma(k, 2.0, sum[i]); t[i] = fma(k, 0.5, xx[i]); }
        ode(p, al, aa, t, d);
#pragma unroll
        for (int i = 0; i < 5; ++i) { const double k = dt * d[i]; sum[i] = fma(k, 2.0, sum[i]); t[i] = xx[i] + k; }
        ode(p, al, aa, t, d);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            s[i] = xx[i] + div6(sum[i] + dt * d[i]);
        }
        if (!BIDIR && s[2] < 0.) s[2] = 0.;
        const double time = s[5] + dt;
        s[5] = time;
        if (s[3] > kPi) s[3] -= 2 * kPi;
        if (s[3] < -kPi) s[3] += 2 * kPi;
        double sn, c;
        sincos_fast(s[3], &sn, &c);
        const double e = get_e(s, c, sn), eph = get_e_phi(s, c, sn);
        int f = 0;  // is_Terminal :247-261
        if (s[0] > p.map_size[0] || s[0] < 0 || s[1] > p.map_size[1] || s[1] < 0) f = 1;
        if (time > p.time_max) f = 2;
        if (fabs(e) <= 0.05 && fabs(s[2]) < 0.01) f = 3;
        obs_from(p, s, e, eph, on);
        const double u_pos = -fabs(e) * p.Q_pos;  // get_reward :263-279
        const double u_vel = -fabs(s[2]) * p.Q_vel;
        const double gate = p.phi_gate_abs ? fabs(e) : e;
        const double u_phi = gate > 0.1 ? -fabs(eph) * p.Q_phi : 0.0;
        const double u_om = -fabs(s[4]) * p.Q_omega;
        double u_psi = 0.;
        if (f == 1) {
            const double n_ = (p.time_max - time) / p.dt;
            u_psi = n_ * (u_pos + u_vel + u_phi + u_om);
        }
        reward = u_pos + u_vel + u_phi + u_om + u_psi;
        flag = f;
        done = f != 0;
    }
    __device__ static __forceinline__ void reset(const P &p, double *s, uint64_t seed,
                                                 uint64_t counter, uint64_t env_id) {
        double u[2], u2[2];  // reset :334-362
        philox_u01_f64x2(seed, counter, env_id, 0x200u, u);
        philox_u01_f64x2(seed, counter, env_id, 0x201u, u2);
        const double d0 = p.reset_margin;
        s[0] = d0 + ((p.map_size[0] - d0) - d0) * u[0];
        s[1] = d0 + ((p.map_size[1] - d0) - d0) * u[1];
        s[3] = -kPi + (kPi - -kPi) * u2[0];
        s[2] = 0.; s[4] = 0.; s[5] = 0.;
        s[6] = p.map_size[0] / 2; s[7] = p.map_size[1] / 2;
    }
};
template <> struct Env<RLP_ENV_UGV_FORWARD> : UGV<false> {};
template <> struct Env<RLP_ENV_UGV_BIDIRECTIONAL> : UGV<true> {};

// ==========================================================================================
// UAV hover outer loop — environment/UavRobust/UavHoverOuterLoop.py (+ uav.py, uav_pos_ctrl.py,
// FNTSMC.py). state: x y z vx vy vz phi theta psi p q r | time | pos_ref[3] | s1[3] | att_ref[3]
// ==========================================================================================
template <> struct Env<RLP_ENV_UAV_HOVER_OUTER_LOOP> {
    using P = rlp_uav_hover_params;
    static constexpr int D = RLP_UAV_D, S = 6, A = 3;
    enum { X = 0, VX = 3, PHI = 6, THE = 7, PSI = 8, PP = 9, T = 12, REF = 13, S1 = 16, AREF = 19 };

    // reciprocals of the step's constant denominators (inertias, mass), shared by the 4 ODE stages
    struct Rc {
        double J[3], m;
    };
    // UAV.ode uav.py:429-460 (J0 = 0, ideal: dis = 0); sc = sin / cos of phi, theta, psi of x
    __device__ static __forceinline__ void ode(const P &p, const Rc &rc, double thr, const double tq[3],
                                               const double *x, const double sc[6], double *d) {
        const double vx = x[3], vy = x[4], vz = x[5];
        const double pp = x[9], q = x[10], r = x[11];
        const double dp = div_r(-p.kr * pp - q * r * (p.J[2] - p.J[1]) + tq[0], p.J[0], rc.J[0]);
        const double dq = div_r(-p.kr * q - pp * r * (p.J[0] - p.J[2]) + tq[1], p.J[1], rc.J[1]);
        const double dr = div_r(-p.kr * r - pp * q * (p.J[1] - p.J[0]) + tq[2], p.J[2], rc.J[2]);
        const double sphi = sc[0], cphi = sc[1], sth = sc[2], cth = sc[3], spsi = sc[4], cpsi = sc[5];
        const double ic = recip_nr(cth);
        const double tth = div_r(sth, cth, ic);
        const double R01 = tth * sphi, R02 = tth * cphi, R11 = cphi, R12 = -sphi;
        const double R21 = div_r(sphi, cth, ic), R22 = div_r(cphi, cth, ic);
        d[6] = 1 * pp + R01 * q + R02 * r;
        d[7] = 0 * pp + R11 * q + R12 * r;
        d[8] = 0 * pp + R21 * q + R22 * r;
        d[0] = vx; d[1] = vy; d[2] = vz;
        d[3] = div_r(thr * (cpsi * sth * cphi + spsi * sphi) - p.kt * vx + 0.0, p.m, rc.m);
        d[4] = div_r(thr * (spsi * sth * cphi - cpsi * sphi) - p.kt * vy + 0.0, p.m, rc.m);
        d[5] = -p.g + div_r(thr * cphi * cth - p.kt * vz + 0.0, p.m, rc.m);
        d[9] = dp; d[10] = dq; d[11] = dr;
    }
    // the stage's angles' sin / cos from the base point's by angle addition (sincos_step)
    __device__ static __forceinline__ void stage_sc(const double sc0[6], const double *s,
                                                    const double *t, double sc[6]) {
#pragma unroll
        for (int i = 0; i < 3; ++i)
            sincos_step(sc0[2 * i], sc0[2 * i + 1], t[PHI + i] - s[PHI + i], &sc[2 * i], &sc[2 * i + 1]);
    }
    __device__ static __forceinline__ void observe(const P &p, const double *s, float *o) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {  // get_state :81-91
            const double e = s[X + i] - s[REF + i];
            o[i] = (float)(e / (p.e_pos_max[i] - p.e_pos_min[i]) * p.static_gain);
            o[3 + i] = (float)(2 * s[VX + i] / (p.vel_max[i] - p.vel_min[i]) * p.static_gain);
        }
    }
    __device__ static __forceinline__ void step(const P &p0, double *s, const float *a, float *on,
                                                double &reward, int &flag, bool &done) {
        const double phi = s[PHI], th = s[THE], psi = s[PSI];
        const double pp = s[PP], q = s[PP + 1], r = s[PP + 2];
        double sphi, cphi, sth, cth, spsi, cpsi;
        sincos_fast(phi, &sphi, &cphi);
        sincos_fast(th, &sth, &cth);
        sincos_fast(psi, &spsi, &cpsi);
        // uo_2_ref_angle_throttle uav_pos_ctrl.py:67-76; (uz + g) * m in float32 (NEP 50)
        const double ux = (double)a[0], uy = (double)a[1];
        const float uzg = (a[2] + (float)p0.g) * (float)p0.m;
        const double uf = div_nr((double)uzg, cphi * cth);
        const double u0 = clipd(div_nr((ux * spsi - uy * cpsi) * p0.m, uf), -1, 1);
        const double phi_d0 = asin(u0);
        double spd, cpd;  // cos(phi_d0) as the reference evaluates it (not sqrt(1 - u0^2))
        sincos_fast(phi_d0, &spd, &cpd);
        const double th_d0 = asin(clipd(div_nr((ux * cpsi + uy * spsi) * p0.m, uf * cpd), -1, 1));
        const double phi_d = clipd(phi_d0, p0.att_zone[0][0], p0.att_zone[0][1]);  // :126-127
        const double th_d = clipd(th_d0, p0.att_zone[1][0], p0.att_zone[1][1]);
        const double aref_new[3] = {phi_d, th_d, 0.0};
        double daref[3], aref[3];
        const double idt = recip_nr(p0.dt);
#pragma unroll
        for (int i = 0; i < 3; ++i) {  // attitude-reference rate limit :130-134
            const double old = s[AREF + i];
            daref[i] = clipd(div_r(aref_new[i] - old, p0.dt, idt), p0.dot_att_min[i], p0.dot_att_max[i]);
            aref[i] = daref[i] * p0.dt + old;
        }
        // att_control uav_pos_ctrl.py:46-65 -> fntsmc_att.control_update FNTSMC.py:80-106
        const P &p = phase_ref(p0);
        const Rc rc = {{recip_nr(p.J[0]), recip_nr(p.J[1]), recip_nr(p.J[2])}, recip_nr(p.m)};
        const double icth = recip_nr(cth);
        const double tth = div_r(sth, cth, icth);
        const double f1[3][3] = {{1., sphi * tth, cphi * tth}, {0., cphi, -sphi},
                                 {0., div_r(sphi, cth, icth), div_r(cphi, cth, icth)}};
        const double rho2[3] = {pp, q, r};
        double drho1[3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
            drho1[i] = f1[i][0] * rho2[0] + f1[i][1] * rho2[1] + f1[i][2] * rho2[2];
        const double f2[3] = {div_r(p.kr * pp + q * r * (p.J[1] - p.J[2]), p.J[0], rc.J[0]),  // uav.py:630-641
                              div_r(p.kr * q + pp * r * (p.J[2] - p.J[0]), p.J[1], rc.J[1]),
                              div_r(p.kr * r + pp * q * (p.J[0] - p.J[1]), p.J[2], rc.J[2])};
        const double c2 = cth * cth, ic2 = recip_nr(c2);  // F uav.py:668-686
        double dF[3][3] = {{0., 0., 0.}, {0., 0., 0.}, {0., 0., 0.}};
        dF[0][1] = drho1[0] * tth * cphi + div_r(drho1[1] * sphi, c2, ic2);
        dF[0][2] = -drho1[0] * tth * sphi + div_r(drho1[1] * cphi, c2, ic2);
        dF[1][1] = -drho1[0] * sphi;
        dF[1][2] = -drho1[0] * cphi;
        dF[2][1] = div_r(drho1[0] * cphi * cth + drho1[1] * sphi * sth, c2, ic2);
        dF[2][2] = div_r(-drho1[0] * sphi * cth + drho1[1] * cphi * sth, c2, ic2);
        const double rho1[3] = {phi, th, psi};
        double u12[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double sec = (dF[i][0] * rho2[0] + dF[i][1] * rho2[1] + dF[i][2] * rho2[2]) +
                               (f1[i][0] * f2[0] + f1[i][1] * f2[1] + f1[i][2] * f2[2]);
            const double e = rho1[i] - aref[i];
            const double de = drho1[i] - daref[i];
            // |e|^alpha and |e|^(alpha-1) from one log: exp(a log|e|) instead of two f64 pow
            // (ocml's pow carries a double-double log for a 1-ulp result; this is within a few
            // ulps, far inside the 1e-9 state parity; pow(0, a) = exp(a * -inf) as pow's)
            const double le = log_fast(fabs(e));
            const double pe = exp_fast(p.att_alpha[i] * le), pe1 = exp_fast((p.att_alpha[i] - 1) * le);
            const double ss = 1 * de + p.att_k1[i] * e + p.att_gamma[i] * pe * tanh_fast(5 * e);
            const double ds1 = exp_fast(p.att_beta[i] * log_fast(fabs(ss))) * tanh_fast(5 * ss);
            s[S1 + i] += ds1 * p.att_ctrl_dt;
            const double sigma = ss + p.att_lmd[i] * s[S1 + i];
            const double u1 = sec + 0.0 + p.att_k1[i] * de +
                              p.att_gamma[i] * p.att_alpha[i] * pe1 * de +
                              p.att_lmd[i] * ds1;
            const double u2 = -p.att_k2[i] * tanh_fast(10 * sigma);
            u12[i] = u1 + u2;
        }
        // -inv(f1 diag(1/J)) (u1+u2) = -diag(J) f1^-1 (u1+u2); f1^-1 of the Euler-rate matrix
        const double fi[3][3] = {{1., 0., -sth}, {0., cphi, sphi * cth}, {0., -sphi, cphi * cth}};
        double tq[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double v = p.J[i] * fi[i][0] * u12[0] + p.J[i] * fi[i][1] * u12[1] +
                             p.J[i] * fi[i][2] * u12[2];
            tq[i] = clipd(-v, -p.att_saturation[i], p.att_saturation[i]);
            s[AREF + i] = aref[i];
        }
        // update -> rk44(n=1) uav.py:462-483
        const double h = p.dt / 1;
        // s[0..11] is the RK4 base point (unchanged until the end); running sum of
        // (K1 + 2*K2 + 2*K3 + K4), bit-identical to the left-to-right expression
        // stage angles' sin / cos: the step's own (stage 1) and angle addition from them (2-4)
        double sum[12], t[12], d[12];
        const double sc0[6] = {sphi, cphi, sth, cth, spsi, cpsi};
        double sc[6];
        ode(phase_ref(p0), rc, uf, tq, s, sc0, d);
#pragma unroll
        for (int i = 0; i < 12; ++i) { const double k = h * d[i]; sum[i] = k; t[i] = fma(k, 0.5, s[i]); }
        stage_sc(sc0, s, t, sc);
        ode(phase_ref(p0), rc, uf, tq, t, sc, d);
#pragma unroll
        for (int i = 0; i < 12; ++i) { const double k = h * d[i]; sum[i] = fma(k, 2.0, sum[i]); t[i] = fma(k, 0.5, s[i]); }
        stage_sc(sc0, s, t, sc);
        ode(phase_ref(p0), rc, uf, tq, t, sc, d);
#pragma unroll
        for (int i = 0; i < 12; ++i) { const double k = h * d[i]; sum[i] = fma(k, 2.0, sum[i]); t[i] = s[i] + k; }
        stage_sc(sc0, s, t, sc);
        ode(phase_ref(p0), rc, uf, tq, t, sc, d);
#pragma unroll
        for (int i = 0; i < 12; ++i) s[i] = s[i] + div6(sum[i] + h * d[i]);
        const P &pr = phase_ref(p0);  // is_episode_Terminal / reward parameters
        s[T] += pr.dt;
        if (s[PSI] > kPi) s[PSI] -= 2 * kPi;
        if (s[PSI] < -kPi) s[PSI] += 2 * kPi;
        int f = 0;  // is_episode_Terminal uav.py:543-560
        if (s[T] > pr.time_max - pr.dt / 2) f = 1;
        bool po = false, ao = false;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            po |= (s[X + i] < pr.pos_zone[i][0]) || (s[X + i] > pr.pos_zone[i][1]);
            ao |= (s[PHI + i] < pr.att_zone[i][0]) || (s[PHI + i] > pr.att_zone[i][1]);
        }
        if (po) f = 2;
        if (ao) f = 3;
        observe(p, s, on);
        // get_reward :93-110; ||x||^2 as the sum of squares (numpy's sqrt-then-square is within
        // 1 ulp of it)
        double nte2 = 0, ne2 = 0, ntv2 = 0, nv2 = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double e = s[X + i] - s[REF + i], v = s[VX + i];
            const double te = tanh_fast(10 * e), tv = tanh_fast(10 * v);
            nte2 += te * te; ne2 += e * e; ntv2 += tv * tv; nv2 += v * v;
        }
        const float na = sqrtf(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);  // float32 action norm
        const double r1 = -nte2 * 0.5 * pr.Qx - ne2 * 0.5 * pr.Qx;
        const double r2 = -ntv2 * 0.5 * pr.Qx - nv2 * 0.5 * pr.Qv;
        const double r3 = (double)(-(na * na) * (float)pr.R);
        double r4 = 0;
        if (po || ao)
            r4 = -div_r(pr.time_max - s[T], pr.dt, idt) *
                 (pr.Qx * ne2 + pr.Qv * nv2 + (double)((float)pr.R * (na * na)));
        reward = r1 + r2 + r3 + r4;
        flag = f;
        done = f != 0;
    }
    // reset(random=True) :152-214; FNTSMC s1 and att_ref are carried over, as in the reference
    __device__ static __forceinline__ void reset(const P &p, double *s, uint64_t seed,
                                                 uint64_t counter, uint64_t env_id) {
        double u[2], u2[2];
        philox_u01_f64x2(seed, counter, env_id, 0x200u, u);
        philox_u01_f64x2(seed, counter, env_id, 0x201u, u2);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            s[X + i] = p.pos0[i]; s[VX + i] = p.vel0[i];
            s[PHI + i] = p.angle0[i]; s[PP + i] = p.pqr0[i];
        }
        s[T] = 0.;
        const double uu[3] = {u[0], u[1], u2[0]};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double lo = p.pos_zone[i][0] + p.target_offset, hi = p.pos_zone[i][1] - p.target_offset;
            s[REF + i] = lo + (hi - lo) * uu[i];
        }
    }
};

// ==========================================================================================
// UGV forward obstacle avoidance — environment/UGVForwardObstacleAvoidance/
// UGVForwardObstacleAvoidance.py. state: x y vel phi omega time tx ty | (cx cy r) x NOBS.
// The fake lidar (get_fake_laser :274-397) is restated in the reference's f64 expression order,
// branch for branch, one env per lane: 37 beams, each against the obstacles in order of distance.
// ==========================================================================================
template <> struct Env<RLP_ENV_UGV_OBSTACLE_AVOIDANCE> {
    using P = rlp_ugv_oa_params;
    static constexpr int NOBS = RLP_UGVOA_NOBS, NL = RLP_UGVOA_NLASER;
    static constexpr int D = RLP_UGVOA_D, S = 4 + NL, A = 2;
    static constexpr int DW = 8;  // step() changes only x..ty (the obstacles are fixed per episode)
    enum { X = 0, Y = 1, V = 2, PHI = 3, OM = 4, T = 5, TX = 6, TY = 7, OB = 8 };

    // utils/functions.py:35-46 cal_vector_rad
    __device__ static __forceinline__ double vec_rad(double x1, double y1, double x2, double y2) {
        const double n1 = sqrt(x1 * x1 + y1 * y1), n2 = sqrt(x2 * x2 + y2 * y2);
        if (n2 < 1e-4 || n1 < 1e-4) return 0;
        double c = (x1 * x2 + y1 * y2) / (n1 * n2);
        c = c > -1 ? c : -1;
        c = c < 1 ? c : 1;
        return acos(c);
    }
    // vec_rad(x1, y1, x2, y2) > pi / 2 (the beam's "obstacle behind the vehicle" test) without the
    // two square roots, the division and the acos where the answer cannot depend on them: with
    // c = cos of the angle, acos(c) > fl(pi / 2) exactly when c < 0 except for |c| below ~1e-16
    // (acos rounds to fl(pi / 2) there), and vec_rad returns 0 (not > pi / 2) for a vector shorter
    // than 1e-4. Outside a relative band of 1e-9 around those thresholds the sign of the dot
    // product decides; inside it the reference's expression runs as written (bit-identical result).
    __device__ static __forceinline__ bool behind(double x1, double y1, double x2, double y2) {
        const double s1 = x1 * x1 + y1 * y1, s2 = x2 * x2 + y2 * y2, dot = x1 * x2 + y1 * y2;
        const bool short_sure = s1 < 1e-8 * (1 - 1e-9) || s2 < 1e-8 * (1 - 1e-9);
        const bool long_sure = s1 > 1e-8 * (1 + 1e-9) && s2 > 1e-8 * (1 + 1e-9);
        if (short_sure) return false;
        if (long_sure && dot * dot > 1e-18 * (s1 * s2)) return dot < 0;  // |c| > 1e-9
        return vec_rad(x1, y1, x2, y2) > kPi / 2;
    }
    // utils/functions.py:49-60 cal_vector_rad_oriented(v1 = [cos phi, sin phi], v2 = target - pos)
    __device__ static __forceinline__ double e_phi(const double *s) {
        const double c = cos(s[PHI]), sn = sin(s[PHI]);
        const double x2 = s[TX] - s[X], y2 = s[TY] - s[Y];
        if (sqrt(x2 * x2 + y2 * y2) < 1e-4 || sqrt(c * c + sn * sn) < 1e-4) return 0;
        return atan2(c * y2 - sn * x2, c * x2 + sn * y2);
    }
    __device__ static __forceinline__ double get_e(const double *s) {  // :512-513
        const double ex = s[TX] - s[X], ey = s[TY] - s[Y];
        return sqrt(ex * ex + ey * ey);
    }
    // collision_check :261-272 over the first n_obs slots; ob(k, x0, y0, r0) fetches obstacle k
    template <class Ob>
    __device__ static __forceinline__ bool collision_at(const P &p, double x, double y, Ob &&ob) {
#pragma unroll
        for (int k = 0; k < NOBS; ++k) {
            if (k >= p.n_obs) continue;
            double x0, y0, r0;
            ob(k, x0, y0, r0);
            const double dx = x - x0, dy = y - y0;
            if (sqrt(dx * dx + dy * dy) <= r0 + p.r_vehicle) return true;
        }
        return false;
    }
    __device__ static __forceinline__ bool collision(const P &p, const double *s) {
        return collision_at(p, s[X], s[Y], [&](int k, double &x0, double &y0, double &r0) {
            x0 = s[OB + 3 * k]; y0 = s[OB + 3 * k + 1]; r0 = s[OB + 3 * k + 2];
        });
    }
    // per-pose part of get_fake_laser: beam angles (np.linspace(phi - R, phi + R, NL): i * step +
    // start, last element = stop) and the four corner angles that pick a beam's wall
    struct Pose {
        double x, y, start, stop, step, th1, th2, th3, th4;
    };
    __device__ static __forceinline__ Pose pose(const P &p, double x, double y, double phi) {
        const double xm = p.map_size[0], ym = p.map_size[1];
        Pose q;
        q.x = x; q.y = y;
        q.start = phi - p.laser_range;
        q.stop = phi + p.laser_range;
        q.step = (q.stop - q.start) / (NL - 1);
        q.th1 = vec_rad(1, 0, xm - x, ym - y);
        q.th2 = vec_rad(1, 0, 0 - x, ym - y);
        q.th3 = -vec_rad(1, 0, 0 - x, 0 - y);
        q.th4 = -vec_rad(1, 0, xm - x, 0 - y);
        return q;
    }
    // beam i of get_fake_laser :283-397 (no collision): distance to the first circle hit, else
    // to the wall / range end. The reference walks the obstacles in argsort(ref_dis) order
    // (stable for <= 16 values) and stops at the first hit; the same result is the hit with the
    // smallest (ref_dis, index), found here without sorting. ob(k, x0, y0, r0, ref) fetches
    // obstacle k and its distance to the vehicle.
    // Two passes: the cheap filters of every obstacle (range, distance of the centre from the beam
    // line) give a candidate mask; the intersection runs for the candidates only. DYN (obstacles
    // in LDS, so a per-lane index is a plain gather): each lane walks its own candidates and a wave
    // iterates max-over-lanes times (a few), instead of NOBS times with the intersection path run
    // whenever any lane of the wave needs it; !DYN (obstacles in a register array) keeps the
    // unrolled walk over compile-time indices.
    // |m x0 - y0 + b| / sq > r0 (the line-distance filter) is decided by a product outside a
    // relative band of 1e-12 and by the reference's division inside it: the same decision.
    template <bool DYN = false, class Ob>
    __device__ static __forceinline__ double beam(const P &p, const Pose &q, int i, Ob &&ob) {
        const double x = q.x, y = q.y, xm = p.map_size[0], ym = p.map_size[1], L = p.laser_dis;
        double ph = i == NL - 1 ? q.stop : (double)i * q.step + q.start;
        if (ph > kPi) ph -= 2 * kPi;
        if (ph < -kPi) ph += 2 * kPi;
        const double m = tan(ph), b = y - m * x;
        const double sq = sqrt(1 + m * m);
        const double cosT = fabs(m) / sq, sinT = 1 / sq;
        double tx, ty;
        if (q.th4 < ph && ph <= q.th1) {
            tx = xm; ty = m * xm + b;
            const double t = x + L / sq;
            if (t < xm) { tx = t; ty = m >= 0 ? y + cosT * L : y - cosT * L; }
        } else if (q.th1 < ph && ph <= q.th2) {
            if (fabs(m) < 1e8) { tx = (ym - b) / m; ty = ym; } else { tx = x; ty = ym; }
            const double t = y + fabs(m) * L / sq;
            if (t < ym) { tx = m >= 0 ? x + L * sinT : x - L * sinT; ty = t; }
        } else if (q.th3 < ph && ph <= q.th4) {
            if (fabs(m) < 1e8) { tx = -b / m; ty = 0; } else { tx = x; ty = 0; }
            const double t = y - fabs(m) * L / sq;
            if (t > 0) { tx = m >= 0 ? x - L * sinT : x + L * sinT; ty = t; }
        } else {
            tx = 0; ty = b;
            const double t = x - L / sq;
            if (t > 0) { tx = t; ty = m >= 0 ? y - cosT * L : y + cosT * L; }
        }
        const double m2 = m * m;
        const double dir = tx - x;
        const double sg = dir > 0 ? 1.0 : (dir < 0 ? -1.0 : 0.0);
        const double lo = x < tx ? x : tx, hi = x < tx ? tx : x;  // min/max(start, terminal)
        bool found = false;
        double val = 0, best = 0;
        unsigned cand = 0;
#pragma unroll
        for (int k = 0; k < NOBS; ++k) {
            if (k >= p.n_obs) continue;
            double x0, y0, r0, ref;
            ob(k, x0, y0, r0, ref);
            if (ref > L + r0) continue;
            const double a = fabs(m * x0 - y0 + b), rs = r0 * sq;
            const bool far = a > rs * (1 + 1e-12) ? true : a < rs * (1 - 1e-12) ? false : a / sq > r0;
            if (!far) cand |= 1u << k;
        }
        auto hit = [&](int k) {  // obstacle k's intersection (the reference's, bit for bit)
            double x0, y0, r0, ref;
            ob(k, x0, y0, r0, ref);
            if (found && !(ref < best)) return;
            if (behind(tx - x, ty - y, x0 - x, y0 - y)) return;
            // (sqrt(m2 + 1) == sq: fl(m * m + 1) is fl(1 + m * m))
            const double fx = (x0 + m * y0 - m * b) / (m2 + 1);
            const double fy = (m * x0 + m2 * y0 + b) / (m2 + 1);
            const double ddx = fx - x0, ddy = fy - y0;
            const double rd = sqrt(ddx * ddx + ddy * ddy);
            const double cross = fx - sg * sqrt(r0 * r0 - rd * rd) / sq;
            if (lo <= cross && cross <= hi) {
                found = true;
                best = ref;
                const double dis = fabs(cross - x) * sq;
                val = dis < p.laser_blind ? p.laser_blind : dis;
            }
        };
        if constexpr (DYN) {
            while (cand) {  // ascending index, as the unrolled walk
                const int k = __builtin_ctz(cand);
                cand &= cand - 1;
                hit(k);
            }
        } else {
#pragma unroll
            for (int k = 0; k < NOBS; ++k)
                if (cand >> k & 1u) hit(k);
        }
        if (!found) {
            const double dx = x - tx, dy = y - ty;
            const double dis = sqrt(dx * dx + dy * dy);
            if (dis > L) val = L;
            else if (p.laser_blind < dis && dis <= L) val = dis;
            else val = p.laser_blind;
        }
        return val;
    }
    // get_state's normalised beam value
    __device__ static __forceinline__ float beam_obs(const P &p, double dis) {
        return (float)((2 * dis / p.laser_dis - 1) * p.static_gain);
    }
    // all beams from the register-resident state (generic env kernels); o[0..NL)
    __device__ static void laser(const P &p, const double *s, float *o) {  // :274-397
        if (collision(p, s)) {
            const float v = beam_obs(p, p.laser_blind);
            for (int i = 0; i < NL; ++i) o[i] = v;
            return;
        }
        double ref[NOBS];
#pragma unroll
        for (int k = 0; k < NOBS; ++k) {
            const double dx = s[X] - s[OB + 3 * k], dy = s[Y] - s[OB + 3 * k + 1];
            ref[k] = sqrt(dx * dx + dy * dy);
        }
        const Pose q = pose(p, s[X], s[Y], s[PHI]);
        for (int i = 0; i < NL; ++i)
            o[i] = beam_obs(p, beam(p, q, i, [&](int k, double &x0, double &y0, double &r0, double &rf) {
                x0 = s[OB + 3 * k]; y0 = s[OB + 3 * k + 1]; r0 = s[OB + 3 * k + 2]; rf = ref[k];
            }));
    }
    __device__ static __forceinline__ void obs_from(const P &p, const double *s, double e,
                                                    double eph, float *o) {  // get_state :399-411
        const double e_max = sqrt(p.map_size[0] * p.map_size[0] + p.map_size[1] * p.map_size[1]) / 2;
        o[0] = (float)((2 / e_max * e - 1) * p.static_gain);
        o[1] = (float)((2 / p.v_max * s[V] - 1) * p.static_gain);
        o[2] = (float)((eph / p.e_phi_max) * p.static_gain);
        o[3] = (float)((s[OM] / p.omega_max) * p.static_gain);
        laser(p, s, o + 4);
    }
    // get_state's first four components (e, vel, e_phi, omega)
    __device__ static __forceinline__ void obs_head(const P &p, const double *s, double e,
                                                    double eph, float *o) {
        const double e_max = sqrt(p.map_size[0] * p.map_size[0] + p.map_size[1] * p.map_size[1]) / 2;
        o[0] = (float)((2 / e_max * e - 1) * p.static_gain);
        o[1] = (float)((2 / p.v_max * s[V] - 1) * p.static_gain);
        o[2] = (float)((eph / p.e_phi_max) * p.static_gain);
        o[3] = (float)((s[OM] / p.omega_max) * p.static_gain);
    }
    __device__ static __forceinline__ void observe(const P &p, const double *s, float *o) {
        obs_from(p, s, get_e(s), e_phi(s), o);
    }
    __device__ static __forceinline__ void ode(const P &p, double al, double aa, const double *x,
                                               double *d) {  // ode :471-482
        d[0] = x[2] * cos(x[3]);
        d[1] = x[2] * sin(x[3]);
        d[2] = al - p.kf * x[2];
        d[3] = x[4];
        d[4] = aa - p.kt * x[4];
    }
    // dynamics, terminal flag and reward of step_update (rk44 -> is_Terminal -> get_reward) on
    // s[0..8); coll(x, y) is collision_check at the new pose. Returns e and e_phi for get_state.
    template <class Coll>
    __device__ static __forceinline__ void step_core(const P &p, double *s, const float *a,
                                                     Coll &&coll, double &reward, int &flag,
                                                     bool &done, double &e_out, double &eph_out) {
        const double al = (double)a[0], aa = (double)a[1], dt = p.dt;
        const double e_max = sqrt(p.map_size[0] * p.map_size[0] + p.map_size[1] * p.map_size[1]) / 2;
        // current_state[0..1] in f64 (the shaped reward compares them with next_state's)
        const double c0 = (2 / e_max * get_e(s) - 1) * p.static_gain;
        const double c1 = (2 / p.v_max * s[V] - 1) * p.static_gain;
        double sum[5], t[5], d[5];  // rk44 :484-502, running RK4 sum (bit-identical, see CartPole)
        ode(p, al, aa, s, d);
#pragma unroll
        for (int i = 0; i < 5; ++i) { const double k = dt * d[i]; sum[i] = k; t[i] = fma(k, 0.5, s[i]); }
        ode(p, al, aa, t, d);
#pragma unroll
        for (int i = 0; i < 5; ++i) { const double k = dt * d[i]; sum[i] = fma(k, 2.0, sum[i]); t[i] = fma(k, 0.5, s[i]); }
        ode(p, al, aa, t, d);
#pragma unroll
        for (int i = 0; i < 5; ++i) { const double k = dt * d[i]; sum[i] = fma(k, 2.0, sum[i]); t[i] = s[i] + k; }
        ode(p, al, aa, t, d);
        if (p.shaped && s[V] < 0.) {  // demo copy rk44 :496-500: gate on the pre-step velocity
            s[PHI] = s[PHI] + div6(sum[PHI] + dt * d[PHI]);
            s[OM] = s[OM] + div6(sum[OM] + dt * d[OM]);
            s[V] = 0.;
        } else {
#pragma unroll
            for (int i = 0; i < 5; ++i) s[i] = s[i] + div6(sum[i] + dt * d[i]);
            if (!p.shaped && s[V] < 0.) s[V] = 0.;
        }
        s[T] = s[T] + dt;
        if (s[PHI] > kPi) s[PHI] -= 2 * kPi;
        if (s[PHI] < -kPi) s[PHI] += 2 * kPi;
        const double e = get_e(s), eph = e_phi(s);
        int f = 0;  // is_Terminal :433-450 (later conditions override)
        if (s[X] > p.map_size[0] || s[X] < 0 || s[Y] > p.map_size[1] || s[Y] < 0) f = 1;
        if (s[T] > p.time_max) f = 2;
        const bool success = fabs(e) <= 0.05 && (p.shaped || fabs(s[OM]) < 0.01) && fabs(s[V]) < 0.01;
        if (success) f = 3;
        if (coll(s[X], s[Y])) f = 4;
        e_out = e;
        eph_out = eph;
        flag = f;
        done = f != 0;
        if (p.shaped) {  // demo copy get_reward :449-473
            const double n0 = (2 / e_max * e - 1) * p.static_gain;
            const double n1 = (2 / p.v_max * s[V] - 1) * p.static_gain;
            const double r1 = -1 - fabs(s[OM]) * 0.1;
            const double r2 = c0 > n0 + 1e-3 ? 5.0 : (1e-3 + c0 < n0 ? -5.0 : 0.0);
            const double r3 = fabs(c1) > fabs(n1) + 1e-2 ? 2.0 : (1e-2 + fabs(c1) < fabs(n1) ? -2.0 : 0.0);
            const double r4 = success ? 500.0 : (f == 4 ? -300.0 : 0.0);
            reward = r1 + r2 + r3 + r4;
            return;
        }
        const double u_pos = -fabs(e) * p.Q_pos;  // get_reward :452-469
        const double u_vel = -fabs(s[V]) * p.Q_vel;
        const double u_phi = e > 0.1 ? -fabs(eph) * p.Q_phi : 0.0;
        const double u_om = -fabs(s[OM]) * p.Q_omega;
        double u_psi = 0.;
        if (f == 1) {
            const double n_ = (p.time_max - s[T]) / p.dt;
            u_psi = n_ * (u_pos + u_vel + u_phi + u_om);
        }
        reward = u_pos + u_vel + u_phi + u_om + u_psi;
    }
    __device__ static void step(const P &p, double *s, const float *a, float *on, double &reward,
                                int &flag, bool &done) {
        double e, eph;
        step_core(p, s, a, [&](double x, double y) {
            return collision_at(p, x, y, [&](int k, double &x0, double &y0, double &r0) {
                x0 = s[OB + 3 * k]; y0 = s[OB + 3 * k + 1]; r0 = s[OB + 3 * k + 2];
            });
        }, reward, flag, done, e, eph);
        obs_from(p, s, e, eph, on);
    }
    // reset(random=True) :520-557 + map.py:66-174 (generate_circle_obs_training). Every draw is
    // Philox-keyed by what it is — (seed, counter, env_id, tag(obstacle k, try t)) — not by how
    // many draws came before, so a wave can test 64 tries of one obstacle at once and keep the
    // first legal one (rlp_lidar.hip oa_reset_kernel) with the same result as this sequential
    // rejection sampler. Requires max_tries <= 65535.
    static constexpr uint32_t kTagStart = 0x40000000u, kTagTarget = 0x41000000u,
                              kTagObs = 0x42000000u, kTagObsR = 0x42800000u, kTagPhi = 0x43000000u;
    // map.py:66-74: U([0.3, 0.3], [xMax - 0.3, yMax - 0.3])
    __device__ static __forceinline__ void draw_point(const P &p, uint64_t seed, uint64_t counter,
                                                      uint64_t id, uint32_t tag, double &x,
                                                      double &y) {
        const double mg = p.st_margin;
        double u[2];
        philox_u01_f64x2(seed, counter, id, tag, u);
        x = mg + ((p.map_size[0] - mg) - mg) * u[0];
        y = mg + ((p.map_size[1] - mg) - mg) * u[1];
    }
    // map.py:76-80: center ~ U([0, 0], [xMax, yMax]), r ~ U(rMin, rMax)
    __device__ static __forceinline__ void draw_obstacle(const P &p, uint64_t seed,
                                                         uint64_t counter, uint64_t id, int k,
                                                         int t, double &cx, double &cy,
                                                         double &r) {
        const uint32_t kt = ((uint32_t)k << 16) + (uint32_t)t;
        double u[2], v[2];
        philox_u01_f64x2(seed, counter, id, kTagObs + kt, u);
        philox_u01_f64x2(seed, counter, id, kTagObsR + kt, v);
        cx = 0 + (p.map_size[0] - 0) * u[0];
        cy = 0 + (p.map_size[1] - 0) * u[1];
        r = p.r_min + (p.r_max - p.r_min) * v[0];
    }
    // map.py:113-127 __is_obs_legal / __is_new_obs_in_obs for a circle against start, target and
    // the k obstacles placed before it (ob(j, x0, y0, r0))
    template <class Ob>
    __device__ static __forceinline__ bool legal(const P &p, double sx, double sy, double tx,
                                                 double ty, double cx, double cy, double r, int k,
                                                 Ob &&ob) {
        double dx = sx - cx, dy = sy - cy;
        if (sqrt(dx * dx + dy * dy) <= r + p.safety_dis_st) return false;
        dx = tx - cx; dy = ty - cy;
        if (sqrt(dx * dx + dy * dy) <= r + p.safety_dis_st) return false;
        bool ok = true;  // every placed obstacle tested (independent square roots, no early exit)
        for (int j = 0; j < k; ++j) {
            double x0, y0, r0;
            ob(j, x0, y0, r0);
            dx = x0 - cx; dy = y0 - cy;
            ok &= !(sqrt(dx * dx + dy * dy) <= r0 + r + p.safety_dis_obs);
        }
        return ok;
    }
    __device__ static __forceinline__ double parked_x(int k) { return -1000.0 - 10.0 * k; }
    static constexpr double kParkedY = -1000.0;
    __device__ static void reset(const P &p, double *s, uint64_t seed, uint64_t counter,
                                 uint64_t env_id) {
        double sx, sy;
        draw_point(p, seed, counter, env_id, kTagStart, sx, sy);
        double tx = sx, ty = sy;  // map.py:68-73: terminal = start; redraw while too close
        for (int t = 0; t < p.max_tries; ++t) {
            const double dx = tx - sx, dy = ty - sy;
            if (sqrt(dx * dx + dy * dy) >= p.safety_dis_st) break;
            draw_point(p, seed, counter, env_id, kTagTarget + (uint32_t)t, tx, ty);
        }
        for (int k = 0; k < NOBS; ++k) {
            double cx = parked_x(k), cy = kParkedY, r = p.r_min;  // parked if unplaceable
            for (int t = 0; k < p.n_obs && t < p.max_tries; ++t) {
                double ccx, ccy, rr;
                draw_obstacle(p, seed, counter, env_id, k, t, ccx, ccy, rr);
                if (legal(p, sx, sy, tx, ty, ccx, ccy, rr, k,
                          [&](int j, double &x0, double &y0, double &r0) {
                              x0 = s[OB + 3 * j]; y0 = s[OB + 3 * j + 1]; r0 = s[OB + 3 * j + 2];
                          })) {
                    cx = ccx; cy = ccy; r = rr;
                    break;
                }
            }
            s[OB + 3 * k] = cx; s[OB + 3 * k + 1] = cy; s[OB + 3 * k + 2] = r;
        }
        double u[2];
        philox_u01_f64x2(seed, counter, env_id, kTagPhi, u);
        s[X] = sx; s[Y] = sy; s[V] = 0.; s[PHI] = -kPi + (kPi - -kPi) * u[0]; s[OM] = 0.;
        s[T] = 0.; s[TX] = tx; s[TY] = ty;
    }
};

// success rule of the driver
__device__ __forceinline__ bool success_of(int rule, int F, bool done, int flag) {
    return rule == RLP_SUCCESS_FLAG_NE ? (flag != F)
         : rule == RLP_SUCCESS_FLAG_EQ ? (flag == F)
                                       : (done && flag != F);
}

}  // namespace rlp
