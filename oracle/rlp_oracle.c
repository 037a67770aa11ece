/*
 * rlp_oracle.c — CPU ORACLE (TEST INFRASTRUCTURE ONLY).
 *
 * Plain-C restatement of the reference's per-env numpy/torch arithmetic for the hot path
 * (HKPolyU-UAV/ReinforcementLearningPlatform). It is the parity checker for librlp.so's HIP
 * kernels and the `cpu_baseline` leg of bench.py — never part of the product path. Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it.
 *
 * Parity pinning: every function is checked in tests/test_oracle_golden.py against golden
 * vectors produced by importing the reference itself (tests/golden/make_golden.py).
 *
 * Arithmetic follows the reference expression by expression (Python left-to-right evaluation,
 * NumPy-2 / NEP-50 promotion: float32 action scalars combined with Python floats stay float32).
 * Compile with -ffp-contract=off so no multiply-add is fused (numpy never fuses).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/rlp.h"

#define PI 3.141592653589793

/* ------------------------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11) — the counter-based RNG the library uses.              */
/* ------------------------------------------------------------------------------------------ */
static void philox4x32_10(uint32_t ctr[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ ctr[1] ^ k0;
        uint32_t n1 = lo1;
        uint32_t n2 = hi0 ^ ctr[3] ^ k1;
        uint32_t n3 = lo0;
        ctr[0] = n0; ctr[1] = n1; ctr[2] = n2; ctr[3] = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

/* block (seed, counter, env_id, purpose|j) -> 4 x u32 */
void oracle_philox_block(uint64_t seed, uint64_t counter, uint64_t env_id, uint32_t tag,
                         uint32_t out[4]) {
    uint32_t c[4];
    c[0] = (uint32_t)counter;
    c[1] = (uint32_t)(counter >> 32) ^ ((uint32_t)(env_id >> 32) << 16);
    c[2] = (uint32_t)env_id;
    c[3] = tag;
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    memcpy(out, c, sizeof(c));
}

/* two uniforms in [0,1) with 53 random bits each */
static void philox_u01_f64x2(uint64_t seed, uint64_t counter, uint64_t env_id, uint32_t tag,
                             double u[2]) {
    uint32_t r[4];
    oracle_philox_block(seed, counter, env_id, tag, r);
    for (int k = 0; k < 2; ++k) {
        uint64_t bits = ((uint64_t)r[2 * k] << 21) ^ (uint64_t)(r[2 * k + 1] >> 11);
        bits &= ((uint64_t)1 << 53) - 1;
        u[k] = (double)bits * (1.0 / 9007199254740992.0);
    }
}

/* Box-Muller pair (fp32) from one block: eps[0], eps[1] (and the 2nd block pair for A > 2) */
void oracle_philox_normal_f32(uint64_t seed, uint64_t counter, uint64_t env_id, int A,
                              float *eps) {
    for (int j = 0; 2 * j < A; ++j) {
        uint32_t r[4];
        oracle_philox_block(seed, counter, env_id, 0x100u + (uint32_t)j, r);
        float u1 = (float)(r[0] >> 8) * 5.9604644775390625e-08f + 2.98023223876953125e-08f;
        float u2 = (float)(r[1] >> 8) * 5.9604644775390625e-08f;
        float rad = sqrtf(-2.0f * logf(u1));
        float th = 6.28318530717958647692f * u2;
        eps[2 * j] = rad * cosf(th);
        if (2 * j + 1 < A) eps[2 * j + 1] = rad * sinf(th);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* CartPole — environment/CartPole/CartPole.py                                                */
/* ------------------------------------------------------------------------------------------ */
static double deg2rad(double d) { return d * PI / 180.; } /* utils/functions.py:4-5 */

/* CartPole.ode :219-238 */
static void cp_ode(const rlp_cartpole_params *p, double force, const double xx[4], double d[4]) {
    double th = xx[0], dth = xx[1], dx = xx[3];
    double S = sin(th), C = cos(th);
    double num = force + p->m * p->ell * (dth * dth) * S;
    num = num - p->kf * dx;
    num = num - 3.0 / 4.0 * p->m * p->g * S * C;
    double den = p->M + p->m - 3.0 / 4.0 * p->m * (C * C);
    double ddx = num / den;
    double ddth = 3.0 / 4.0 / p->m / p->ell * (p->m * p->g * S - p->m * ddx * C);
    d[0] = dth;
    d[1] = ddth;
    d[2] = dx;
    d[3] = ddx;
}

/* CartPole.get_state :145-153 */
static void cp_obs(const rlp_cartpole_params *p, const double *s, float *o) {
    o[0] = (float)((s[0] / p->theta_max) * p->static_gain);
    o[1] = (float)((s[1] / p->dtheta_max) * p->static_gain);
    o[2] = (float)((s[2] / p->x_max) * p->static_gain);
    o[3] = (float)((s[3] / p->dx_max) * p->static_gain);
}

/* CartPole.step_update :257-264 = get_state, rk44 :240-255, is_Terminal :160-185,
 * get_state, get_reward :187-217. s = {theta, dtheta, x, dx, time}. */
static void cp_step(const rlp_cartpole_params *p, double *s, float a, float *obs_cur,
                    float *obs_next, double *reward, int32_t *flag, uint8_t *done) {
    if (obs_cur) cp_obs(p, s, obs_cur);
    double force = (double)a;
    double h = p->dt / (double)p->n_sub_div;
    double time = s[4];
    double tt = time + p->dt;
    double xx[4] = {s[0], s[1], s[2], s[3]};
    while (time < tt) {
        double K1[4], K2[4], K3[4], K4[4], tmp[4], d[4];
        cp_ode(p, force, xx, d);
        for (int i = 0; i < 4; ++i) K1[i] = h * d[i];
        for (int i = 0; i < 4; ++i) tmp[i] = xx[i] + K1[i] / 2;
        cp_ode(p, force, tmp, d);
        for (int i = 0; i < 4; ++i) K2[i] = h * d[i];
        for (int i = 0; i < 4; ++i) tmp[i] = xx[i] + K2[i] / 2;
        cp_ode(p, force, tmp, d);
        for (int i = 0; i < 4; ++i) K3[i] = h * d[i];
        for (int i = 0; i < 4; ++i) tmp[i] = xx[i] + K3[i];
        cp_ode(p, force, tmp, d);
        for (int i = 0; i < 4; ++i) K4[i] = h * d[i];
        for (int i = 0; i < 4; ++i) xx[i] = xx[i] + (K1[i] + 2 * K2[i] + 2 * K3[i] + K4[i]) / 6;
        time += h;
    }
    s[0] = xx[0]; s[1] = xx[1]; s[2] = xx[2]; s[3] = xx[3]; s[4] = time;
    double th = s[0], dth = s[1], x = s[2], dx = s[3];
    double eth = 0. - th, ex = 0. - x;
    /* is_Terminal (note the reference's asymmetric lower bound uses dtheta_max, :167) */
    int f = 0;
    uint8_t term = 0;
    if ((th > p->theta_max + deg2rad(1)) || th < -p->dtheta_max - deg2rad(1)) { f = 1; term = 1; }
    if (x > p->x_max || x < -p->x_max) { f = 2; term = 1; }
    if (time > p->time_max) { f = 3; term = 1; }
    if (sqrt(ex * ex + dx * dx + eth * eth + dth * dth) < 1e-2) { f = 4; term = 1; }
    cp_obs(p, s, obs_next);
    /* get_reward; r_f is float32 arithmetic under NEP 50 (np.float32 force * Python float) */
    double r_x = -fabs(x) * p->Q_x;
    double r_dx = -fabs(dx) * p->Q_dx;
    double r_th = -fabs(th) * p->Q_theta;
    double r_om = -fabs(dth) * p->Q_omega;
    float r_f32 = -fabsf(a) * (float)p->R;
    double r_f = (double)r_f32;
    double r_extra = 0.;
    if (f == 1 || f == 2) {
        double n_ = (p->time_max - time) / p->dt;
        r_extra = n_ * (r_x + r_dx + r_th + r_om + r_f);
    }
    *reward = r_x + r_dx + r_th + r_om + r_f + r_extra;
    *flag = f;
    *done = term;
}

/* ------------------------------------------------------------------------------------------ */
/* CartPoleAngleOnly — demonstration/PPO2/PPO2-4-CartPoleAngleOnly/cartpole_angleonly.py       */
/* ------------------------------------------------------------------------------------------ */
static void ao_ode(const rlp_angleonly_params *p, double force, const double xx[4], double d[4]) {
    double th = xx[0], dth = xx[1], dx = xx[3];
    double S = sin(th), C = cos(th);
    double num = force + p->m * p->ell * (dth * dth) * S;
    num = num - p->kf * dx;
    num = num - 3.0 / 4.0 * p->m * p->g * S * C;
    double den = p->M + p->m - 3.0 / 4.0 * p->m * (C * C);
    double ddx = num / den;
    double ddth = 3.0 / 4.0 / p->m / p->ell * (p->m * p->g * S - p->m * ddx * C);
    d[0] = dth; d[1] = ddth; d[2] = dx; d[3] = ddx;
}

static void ao_obs(const rlp_angleonly_params *p, const double *s, float *o) { /* :137-143 */
    o[0] = (float)((s[0] / p->theta_max) * p->static_gain);
    o[1] = (float)((s[1] / p->norm_dtheta) * p->static_gain);
}

static void ao_rk4(const rlp_angleonly_params *p, double force, double h, double xx[4]) {
    double K1[4], K2[4], K3[4], K4[4], tmp[4], d[4];
    ao_ode(p, force, xx, d);
    for (int i = 0; i < 4; ++i) K1[i] = h * d[i];
    for (int i = 0; i < 4; ++i) tmp[i] = xx[i] + K1[i] / 2;
    ao_ode(p, force, tmp, d);
    for (int i = 0; i < 4; ++i) K2[i] = h * d[i];
    for (int i = 0; i < 4; ++i) tmp[i] = xx[i] + K2[i] / 2;
    ao_ode(p, force, tmp, d);
    for (int i = 0; i < 4; ++i) K3[i] = h * d[i];
    for (int i = 0; i < 4; ++i) tmp[i] = xx[i] + K3[i];
    ao_ode(p, force, tmp, d);
    for (int i = 0; i < 4; ++i) K4[i] = h * d[i];
    for (int i = 0; i < 4; ++i) xx[i] = xx[i] + (K1[i] + 2 * K2[i] + 2 * K3[i] + K4[i]) / 6;
}

/* |rad2deg(current_state[0] / staticGain * thetaMax)| (environment/CartPole/
 * CartPoleAngleOnly.py:187-188; rad2deg = deg * 180. / pi, utils/functions.py:8-9) */
static double ao_abs_deg(const rlp_angleonly_params *p, double th) {
    double o = th / p->theta_max * p->static_gain;
    return fabs(o / p->static_gain * p->theta_max * 180. / PI);
}

static void ao_step(const rlp_angleonly_params *p, double *s, float a, float *obs_cur,
                    float *obs_next, double *reward, int32_t *flag, uint8_t *done) {
    if (obs_cur) ao_obs(p, s, obs_cur);
    double force = (double)a;
    double xx[4] = {s[0], s[1], s[2], s[3]};
    double th0 = s[0];
    double time = s[4];
    if (p->variant == RLP_ANGLEONLY_ENV_FILE) { /* env file rk44 :231-244 */
        double h = p->dt / (double)p->n_sub_div, tt = time + p->dt;
        while (time < tt) {
            ao_rk4(p, force, h, xx);
            time += h;
        }
    } else { /* PPO2 copy rk44 :218-229, one step of dt */
        ao_rk4(p, force, p->dt, xx);
        time = s[4] + p->dt;
    }
    s[0] = xx[0]; s[1] = xx[1]; s[2] = xx[2]; s[3] = xx[3]; s[4] = time;
    double th = s[0], dth = s[1];
    double eth = 0. - th;
    int f = 0;
    uint8_t term = 0;
    int out = (th > p->theta_max + deg2rad(1)) || th < -p->theta_max - deg2rad(1);
    ao_obs(p, s, obs_next);
    if (p->variant == RLP_ANGLEONLY_ENV_FILE) {
        /* is_Terminal :144-166 (angle first, returns early; no success flag) */
        if (out) f = 1;
        else if (time > p->time_max) f = 3;
        term = f != 0;
        /* get_reward :168-208 */
        double cur = ao_abs_deg(p, th0), nex = ao_abs_deg(p, th);
        double r;
        if (nex > cur) r = -2;
        else if (nex == cur) r = 0;
        else r = 2;
        if (cur <= 0.5 && nex <= 0.5) r += 5;
        if (f == 1) r -= 100;
        else if (f == 3) r += 500;
        *reward = r;
    } else {
        if (out) { f = 1; term = 1; }
        if (time > p->time_max) { f = 3; term = 1; }
        if (sqrt(eth * eth + dth * dth) < 1e-2) { f = 4; term = 1; }
        /* get_reward :170-195 (r3 in float32: np.float32 force) */
        double r1 = -(th * th) * p->Q_theta;
        double r2 = -(dth * dth) * p->Q_omega;
        float r3f = -(a * a) * (float)p->R;
        double r3 = (double)r3f;
        double r4 = 0.;
        if (f == 1) {
            double n_ = (p->time_max - time) / p->dt;
            r4 = n_ * (r1 + r2 + r3);
        }
        *reward = r1 + r2 + r3 + r4;
    }
    *flag = f;
    *done = term;
}

/* ------------------------------------------------------------------------------------------ */
/* SecondOrderIntegration — environment/SecondOrderIntegration/SecondOrderIntegration.py      */
/* s = {x, y, vx, vy, time, tx, ty}                                                           */
/* ------------------------------------------------------------------------------------------ */
static void soi_obs(const rlp_soi_params *p, const double *s, float *o) { /* :211-219 */
    double ex = s[5] - s[0], ey = s[6] - s[1];
    o[0] = (float)((ex / p->map_size[0]) * p->obs_gain);
    o[1] = (float)((ey / p->map_size[1]) * p->obs_gain);
    o[2] = (float)((-s[2] / p->v_max) * p->obs_gain);
    o[3] = (float)((-s[3] / p->v_max) * p->obs_gain);
}

static void soi_step(const rlp_soi_params *p, double *s, const float *a, float *obs_cur,
                     float *obs_next, double *reward, int32_t *flag, uint8_t *done) {
    if (obs_cur) soi_obs(p, s, obs_cur);
    double f0 = (double)a[0], f1 = (double)a[1];
    double h = p->dt / 1;
    double time = s[4];
    double tt = time + p->dt;
    while (time < tt) { /* rk44 :298-314 */
        double xx[4] = {s[0], s[1], s[2], s[3]};
        double K1[4], K2[4], K3[4], K4[4], t[4];
        K1[0] = h * xx[2]; K1[1] = h * xx[3];
        K1[2] = h * (f0 - p->k * xx[2]); K1[3] = h * (f1 - p->k * xx[3]);
        for (int i = 0; i < 4; ++i) t[i] = xx[i] + K1[i] / 2;
        K2[0] = h * t[2]; K2[1] = h * t[3];
        K2[2] = h * (f0 - p->k * t[2]); K2[3] = h * (f1 - p->k * t[3]);
        for (int i = 0; i < 4; ++i) t[i] = xx[i] + K2[i] / 2;
        K3[0] = h * t[2]; K3[1] = h * t[3];
        K3[2] = h * (f0 - p->k * t[2]); K3[3] = h * (f1 - p->k * t[3]);
        for (int i = 0; i < 4; ++i) t[i] = xx[i] + K3[i];
        K4[0] = h * t[2]; K4[1] = h * t[3];
        K4[2] = h * (f0 - p->k * t[2]); K4[3] = h * (f1 - p->k * t[3]);
        for (int i = 0; i < 4; ++i) s[i] = xx[i] + (K1[i] + 2 * K2[i] + 2 * K3[i] + K4[i]) / 6;
        time += h;
    }
    s[4] = time;
    double accx = (f0 - p->k * s[2]) / p->mass, accy = (f1 - p->k * s[3]) / p->mass;
    double ex = s[5] - s[0], ey = s[6] - s[1];
    int f = 0;
    uint8_t term = 0;
    double adm = p->admissible_error;
    if (s[0] > p->map_size[0] + adm || s[0] < 0 - adm || s[1] > p->map_size[1] + adm ||
        s[1] < 0 - adm) { f = 1; term = 1; }
    if (time > p->time_max) { f = 2; term = 1; }
    if (p->success_enabled && sqrt(ex * ex + ey * ey) <= 0.05 &&
        sqrt(s[2] * s[2] + s[3] * s[3]) < 0.05) { f = 3; term = 1; }
    soi_obs(p, s, obs_next);
    double e_pos = sqrt(ex * ex + ey * ey); /* get_reward :251-284 */
    double e_vel = sqrt(s[2] * s[2] + s[3] * s[3]);
    double acc = sqrt(accx * accx + accy * accy);
    double u_pos = -e_pos * p->Q_pos, u_vel = -e_vel * p->Q_vel, u_acc = -acc * p->Q_acc;
    double u_extra = 0.;
    if (f == 1) {
        double n_ = (p->time_max - time) / p->dt;
        u_extra = n_ * (u_pos + u_vel + u_acc);
    }
    *reward = u_pos + u_vel + u_acc + u_extra;
    *flag = f;
    *done = term;
}

/* ------------------------------------------------------------------------------------------ */
/* UGVForward / UGVBidirectional — environment/UGV/UGVForward.py, UGVBidirectional.py         */
/* s = {x, y, vel, phi, omega, time, tx, ty}                                                  */
/* ------------------------------------------------------------------------------------------ */
static double ugv_e(int bidir, const double *s) { /* get_e :315-317 / Bidir :315-319 */
    double ex = s[6] - s[0], ey = s[7] - s[1];
    double v = sqrt(ex * ex + ey * ey);
    if (!bidir) return v;
    double dot = cos(s[3]) * ex + sin(s[3]) * ey;
    double sg = dot > 0 ? 1.0 : (dot < 0 ? -1.0 : 0.0);
    return sg * v;
}

static double ugv_ephi(int bidir, const double *s) { /* get_e_phi -> cal_vector_rad_oriented */
    double x1 = cos(s[3]), y1 = sin(s[3]);
    double x2 = s[6] - s[0], y2 = s[7] - s[1];
    double ph;
    if (sqrt(x2 * x2 + y2 * y2) < 1e-4 || sqrt(x1 * x1 + y1 * y1) < 1e-4) {
        ph = 0;
    } else {
        double dot = x1 * x2 + y1 * y2;
        double det = x1 * y2 - y1 * x2;
        ph = atan2(det, dot);
    }
    if (bidir) {
        ph = ph >= PI / 2 ? ph - PI : ph;
        ph = ph <= -PI / 2 ? ph + PI : ph;
    }
    return ph;
}

static void ugv_obs(const rlp_ugv_params *p, int bidir, const double *s, float *o) {
    double e = ugv_e(bidir, s), eph = ugv_ephi(bidir, s);
    double e_max = sqrt(p->map_size[0] * p->map_size[0] + p->map_size[1] * p->map_size[1]) / 2;
    double s0, s1;
    if (!bidir) {
        s0 = 2 / e_max * e - 1;
        s1 = 2 / p->v_max * s[2] - 1;
    } else {
        s0 = e / e_max;
        s1 = s[2] / p->v_max;
    }
    o[0] = (float)(s0 * p->static_gain);
    o[1] = (float)(s1 * p->static_gain);
    o[2] = (float)((eph / PI) * p->static_gain);
    o[3] = (float)((s[4] / p->omega_max) * p->static_gain);
}

static void ugv_ode(const rlp_ugv_params *p, double al, double aa, const double *x, double *d) {
    d[0] = x[2] * cos(x[3]);
    d[1] = x[2] * sin(x[3]);
    d[2] = al - p->kf * x[2];
    d[3] = x[4];
    d[4] = aa - p->kt * x[4];
}

static void ugv_step(const rlp_ugv_params *p, int bidir, double *s, const float *a,
                     float *obs_cur, float *obs_next, double *reward, int32_t *flag,
                     uint8_t *done) {
    if (obs_cur) ugv_obs(p, bidir, s, obs_cur);
    double al = (double)a[0], aa = (double)a[1];
    double xx[5] = {s[0], s[1], s[2], s[3], s[4]};
    double K1[5], K2[5], K3[5], K4[5], t[5], d[5];
    double dt = p->dt;
    ugv_ode(p, al, aa, xx, d);
    for (int i = 0; i < 5; ++i) K1[i] = dt * d[i];
    for (int i = 0; i < 5; ++i) t[i] = xx[i] + K1[i] / 2;
    ugv_ode(p, al, aa, t, d);
    for (int i = 0; i < 5; ++i) K2[i] = dt * d[i];
    for (int i = 0; i < 5; ++i) t[i] = xx[i] + K2[i] / 2;
    ugv_ode(p, al, aa, t, d);
    for (int i = 0; i < 5; ++i) K3[i] = dt * d[i];
    for (int i = 0; i < 5; ++i) t[i] = xx[i] + K3[i];
    ugv_ode(p, al, aa, t, d);
    for (int i = 0; i < 5; ++i) K4[i] = dt * d[i];
    for (int i = 0; i < 5; ++i) xx[i] = xx[i] + (K1[i] + 2 * K2[i] + 2 * K3[i] + K4[i]) / 6;
    s[0] = xx[0]; s[1] = xx[1]; s[2] = xx[2]; s[3] = xx[3]; s[4] = xx[4];
    if (!bidir && s[2] < 0.) s[2] = 0.;
    double time = s[5] + dt;
    s[5] = time;
    if (s[3] > PI) s[3] -= 2 * PI;
    if (s[3] < -PI) s[3] += 2 * PI;
    double e = ugv_e(bidir, s), eph = ugv_ephi(bidir, s);
    int f = 0;
    uint8_t term = 0;
    if (s[0] > p->map_size[0] || s[0] < 0 || s[1] > p->map_size[1] || s[1] < 0) { f = 1; term = 1; }
    if (time > p->time_max) { f = 2; term = 1; }
    if (fabs(e) <= 0.05 && fabs(s[2]) < 0.01) { f = 3; term = 1; }
    ugv_obs(p, bidir, s, obs_next);
    double u_pos = -fabs(e) * p->Q_pos;
    double u_vel = -fabs(s[2]) * p->Q_vel;
    double gate = p->phi_gate_abs ? fabs(e) : e;
    double u_phi = gate > 0.1 ? -fabs(eph) * p->Q_phi : 0.0;
    double u_om = -fabs(s[4]) * p->Q_omega;
    double u_psi = 0.;
    if (f == 1) {
        double n_ = (p->time_max - time) / p->dt;
        u_psi = n_ * (u_pos + u_vel + u_phi + u_om);
    }
    *reward = u_pos + u_vel + u_phi + u_om + u_psi;
    *flag = f;
    *done = term;
}

/* ------------------------------------------------------------------------------------------ */
/* UAV hover outer loop — environment/UavRobust/{UavHoverOuterLoop,uav,uav_pos_ctrl,FNTSMC}.py */
/* s = {x y z vx vy vz phi theta psi p q r | time | ref[3] | s1[3] | att_ref[3]}              */
/* ------------------------------------------------------------------------------------------ */
enum { U_X = 0, U_VX = 3, U_PHI = 6, U_THE = 7, U_PSI = 8, U_P = 9, U_T = 12, U_REF = 13,
       U_S1 = 16, U_AREF = 19 };

/* UAV.ode uav.py:429-460 (J0 = 0, dis = 0) */
static void uav_ode(const rlp_uav_hover_params *p, double thr, const double tq[3],
                    const double *x, double *d) {
    double vx = x[3], vy = x[4], vz = x[5], phi = x[6], th = x[7], psi = x[8];
    double pp = x[9], q = x[10], r = x[11];
    const double *J = p->J;
    double dp = (-p->kr * pp - q * r * (J[2] - J[1]) + tq[0]) / J[0];
    double dq = (-p->kr * q - pp * r * (J[0] - J[2]) + tq[1]) / J[1];
    double dr = (-p->kr * r - pp * q * (J[1] - J[0]) + tq[2]) / J[2];
    double R00 = 1, R01 = tan(th) * sin(phi), R02 = tan(th) * cos(phi);
    double R10 = 0, R11 = cos(phi), R12 = -sin(phi);
    double R20 = 0, R21 = sin(phi) / cos(th), R22 = cos(phi) / cos(th);
    double dphi = R00 * pp + R01 * q + R02 * r;
    double dth = R10 * pp + R11 * q + R12 * r;
    double dpsi = R20 * pp + R21 * q + R22 * r;
    double dvx = (thr * (cos(psi) * sin(th) * cos(phi) + sin(psi) * sin(phi)) - p->kt * vx + 0.0) / p->m;
    double dvy = (thr * (sin(psi) * sin(th) * cos(phi) - cos(psi) * sin(phi)) - p->kt * vy + 0.0) / p->m;
    double dvz = -p->g + (thr * cos(phi) * cos(th) - p->kt * vz + 0.0) / p->m;
    d[0] = vx; d[1] = vy; d[2] = vz; d[3] = dvx; d[4] = dvy; d[5] = dvz;
    d[6] = dphi; d[7] = dth; d[8] = dpsi; d[9] = dp; d[10] = dq; d[11] = dr;
}

static void uav_obs(const rlp_uav_hover_params *p, const double *s, float *o) { /* :81-91 */
    for (int i = 0; i < 3; ++i) {
        double e = s[U_X + i] - s[U_REF + i];
        o[i] = (float)(e / (p->e_pos_max[i] - p->e_pos_min[i]) * p->static_gain);
        o[3 + i] = (float)(2 * s[U_VX + i] / (p->vel_max[i] - p->vel_min[i]) * p->static_gain);
    }
}

static int uav_pos_out(const rlp_uav_hover_params *p, const double *s) { /* uav.py:511-525 */
    int f = 0;
    for (int i = 0; i < 3; ++i)
        if (s[U_X + i] < p->pos_zone[i][0] || s[U_X + i] > p->pos_zone[i][1]) f = 1;
    return f;
}
static int uav_att_out(const rlp_uav_hover_params *p, const double *s) { /* uav.py:527-541 */
    int f = 0;
    for (int i = 0; i < 3; ++i)
        if (s[U_PHI + i] < p->att_zone[i][0] || s[U_PHI + i] > p->att_zone[i][1]) f = 1;
    return f;
}
static double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
static double sgn_tanh(double x) { return tanh(x); }

static void uav_step(const rlp_uav_hover_params *p, double *s, const float *a, float *obs_cur,
                     float *obs_next, double *reward, int32_t *flag, uint8_t *done) {
    if (obs_cur) uav_obs(p, s, obs_cur);
    double phi = s[U_PHI], th = s[U_THE], psi = s[U_PSI];
    double pp = s[U_P], q = s[U_P + 1], r = s[U_P + 2];
    /* uo_2_ref_angle_throttle uav_pos_ctrl.py:67-76 ((uz + g) * m is float32 under NEP 50) */
    double ux = (double)a[0], uy = (double)a[1];
    float uzg = (a[2] + (float)p->g) * (float)p->m;
    double uf = (double)uzg / (cos(phi) * cos(th));
    double asin_phi = clipd((ux * sin(psi) - uy * cos(psi)) * p->m / uf, -1, 1);
    double phi_d = asin(asin_phi);
    double asin_th = clipd((ux * cos(psi) + uy * sin(psi)) * p->m / (uf * cos(phi_d)), -1, 1);
    double th_d = asin(asin_th);
    phi_d = clipd(phi_d, p->att_zone[0][0], p->att_zone[0][1]); /* UavHoverOuterLoop.py:126-127 */
    th_d = clipd(th_d, p->att_zone[1][0], p->att_zone[1][1]);
    /* attitude reference rate limit :130-134 */
    double aref_old[3] = {s[U_AREF], s[U_AREF + 1], s[U_AREF + 2]};
    double aref_new[3] = {phi_d, th_d, 0.0};
    double daref[3], aref[3];
    for (int i = 0; i < 3; ++i) {
        daref[i] = (aref_new[i] - aref_old[i]) / p->dt;
        daref[i] = clipd(daref[i], p->dot_att_min[i], p->dot_att_max[i]);
        aref[i] = daref[i] * p->dt + aref_old[i];
    }
    /* att_control uav_pos_ctrl.py:46-65 -> fntsmc_att.control_update FNTSMC.py:80-106 */
    double sphi = sin(phi), cphi = cos(phi), tth = tan(th), cth = cos(th), sth = sin(th);
    double f1[3][3] = {{1., sphi * tth, cphi * tth}, {0., cphi, -sphi}, {0., sphi / cth, cphi / cth}};
    double rho2[3] = {pp, q, r};
    double drho1[3];
    for (int i = 0; i < 3; ++i) drho1[i] = f1[i][0] * rho2[0] + f1[i][1] * rho2[1] + f1[i][2] * rho2[2];
    const double *J = p->J;
    double f2[3] = {(p->kr * pp + q * r * (J[1] - J[2])) / J[0],
                    (p->kr * q + pp * r * (J[2] - J[0])) / J[1],
                    (p->kr * r + pp * q * (J[0] - J[1])) / J[2]}; /* uav.py:630-641 */
    double dF[3][3] = {{0}};                                             /* F uav.py:668-686 */
    dF[0][1] = drho1[0] * tth * cphi + drho1[1] * sphi / (cth * cth);
    dF[0][2] = -drho1[0] * tth * sphi + drho1[1] * cphi / (cth * cth);
    dF[1][1] = -drho1[0] * sphi;
    dF[1][2] = -drho1[0] * cphi;
    double t1 = drho1[0] * cphi * cth + drho1[1] * sphi * sth;
    dF[2][1] = t1 / (cth * cth);
    double t2 = -drho1[0] * sphi * cth + drho1[1] * cphi * sth;
    dF[2][2] = t2 / (cth * cth);
    double sec[3];
    for (int i = 0; i < 3; ++i) {
        double a1 = dF[i][0] * rho2[0] + dF[i][1] * rho2[1] + dF[i][2] * rho2[2];
        double a2 = f1[i][0] * f2[0] + f1[i][1] * f2[1] + f1[i][2] * f2[2];
        sec[i] = a1 + a2;
    }
    double rho1[3] = {phi, th, psi};
    double u12[3];
    for (int i = 0; i < 3; ++i) {
        double e = rho1[i] - aref[i];
        double de = drho1[i] - daref[i];
        double ss = 1 * de + p->att_k1[i] * e + p->att_gamma[i] * pow(fabs(e), p->att_alpha[i]) * sgn_tanh(5 * e);
        double ds1 = pow(fabs(ss), p->att_beta[i]) * sgn_tanh(5 * ss);
        s[U_S1 + i] += ds1 * p->att_ctrl_dt;
        double sigma = ss + p->att_lmd[i] * s[U_S1 + i];
        double u1 = sec[i] + 0.0 + p->att_k1[i] * de +
                    p->att_gamma[i] * p->att_alpha[i] * pow(fabs(e), p->att_alpha[i] - 1) * de +
                    p->att_lmd[i] * ds1;
        double u2 = -p->att_k2[i] * sgn_tanh(10 * sigma);
        u12[i] = u1 + u2;
    }
    /* control = -inv(f1 * diag(1/J)) (u1 + u2) = -diag(J) f1^-1 (u1 + u2); closed-form inverse of
       the Euler-rate matrix: [[1,0,-s(th)],[0,c(phi),s(phi)c(th)],[0,-s(phi),c(phi)c(th)]] */
    double fi[3][3] = {{1., 0., -sth}, {0., cphi, sphi * cth}, {0., -sphi, cphi * cth}};
    double tq[3];
    for (int i = 0; i < 3; ++i) {
        double v = J[i] * fi[i][0] * u12[0] + J[i] * fi[i][1] * u12[1] + J[i] * fi[i][2] * u12[2];
        tq[i] = clipd(-v, -p->att_saturation[i], p->att_saturation[i]);
    }
    for (int i = 0; i < 3; ++i) s[U_AREF + i] = aref[i];
    /* update -> rk44(n=1) uav.py:462-483 */
    double h = p->dt / 1;
    double xx[12], K1[12], K2[12], K3[12], K4[12], t[12], d[12];
    for (int i = 0; i < 12; ++i) xx[i] = s[i];
    uav_ode(p, uf, tq, xx, d);
    for (int i = 0; i < 12; ++i) K1[i] = h * d[i];
    for (int i = 0; i < 12; ++i) t[i] = xx[i] + K1[i] / 2;
    uav_ode(p, uf, tq, t, d);
    for (int i = 0; i < 12; ++i) K2[i] = h * d[i];
    for (int i = 0; i < 12; ++i) t[i] = xx[i] + K2[i] / 2;
    uav_ode(p, uf, tq, t, d);
    for (int i = 0; i < 12; ++i) K3[i] = h * d[i];
    for (int i = 0; i < 12; ++i) t[i] = xx[i] + K3[i];
    uav_ode(p, uf, tq, t, d);
    for (int i = 0; i < 12; ++i) K4[i] = h * d[i];
    for (int i = 0; i < 12; ++i) s[i] = xx[i] + (K1[i] + 2 * K2[i] + 2 * K3[i] + K4[i]) / 6;
    s[U_T] += p->dt;
    if (s[U_PSI] > PI) s[U_PSI] -= 2 * PI;
    if (s[U_PSI] < -PI) s[U_PSI] += 2 * PI;
    /* is_episode_Terminal uav.py:543-560 */
    int f = 0;
    uint8_t term = 0;
    if (s[U_T] > p->time_max - p->dt / 2) { f = 1; term = 1; }
    int po = uav_pos_out(p, s), ao = uav_att_out(p, s);
    if (po) { f = 2; term = 1; }
    if (ao) { f = 3; term = 1; }
    uav_obs(p, s, obs_next);
    /* get_reward UavHoverOuterLoop.py:93-110 (action norm in float32) */
    double e[3], v[3];
    for (int i = 0; i < 3; ++i) { e[i] = s[U_X + i] - s[U_REF + i]; v[i] = s[U_VX + i]; }
    double nte = 0, ne = 0, ntv = 0, nv = 0;
    for (int i = 0; i < 3; ++i) {
        double te = tanh(10 * e[i]), tv = tanh(10 * v[i]);
        nte += te * te; ne += e[i] * e[i]; ntv += tv * tv; nv += v[i] * v[i];
    }
    nte = sqrt(nte); ne = sqrt(ne); ntv = sqrt(ntv); nv = sqrt(nv);
    float na = sqrtf(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    double r1 = -(nte * nte) * 0.5 * p->Qx - ne * ne * 0.5 * p->Qx;
    double r2 = -(ntv * ntv) * 0.5 * p->Qx - nv * nv * 0.5 * p->Qv;
    float r3f = -(na * na) * (float)p->R;
    double r3 = (double)r3f;
    double r4 = 0;
    if (po || ao) {
        float ra = (float)p->R * (na * na);
        r4 = -(p->time_max - s[U_T]) / p->dt * (p->Qx * (ne * ne) + p->Qv * (nv * nv) + (double)ra);
    }
    *reward = r1 + r2 + r3 + r4;
    *flag = f;
    *done = term;
}

/* ------------------------------------------------------------------------------------------ */
/* UGV forward obstacle avoidance — environment/UGVForwardObstacleAvoidance/                  */
/* UGVForwardObstacleAvoidance.py. s = {x y vel phi omega time tx ty | (cx cy r) x NOBS}       */
/* ------------------------------------------------------------------------------------------ */
#define OA_NOBS RLP_UGVOA_NOBS
#define OA_NL RLP_UGVOA_NLASER

static double oa_vec_rad(double x1, double y1, double x2, double y2) { /* functions.py:35-46 */
    double n1 = sqrt(x1 * x1 + y1 * y1), n2 = sqrt(x2 * x2 + y2 * y2);
    if (n2 < 1e-4 || n1 < 1e-4) return 0;
    double c = (x1 * x2 + y1 * y2) / (n1 * n2);
    return acos(fmin(fmax(c, -1.0), 1.0));
}

static double oa_dis(double x1, double y1, double x2, double y2) { /* dis_two_points */
    double dx = x1 - x2, dy = y1 - y2;
    return sqrt(dx * dx + dy * dy);
}

/* obstacle slots >= n_obs are not part of the map (reset parks them outside it) */
static int oa_collision(const rlp_ugv_oa_params *p, const double *s) { /* :261-272 */
    for (int k = 0; k < p->n_obs; ++k)
        if (oa_dis(s[0], s[1], s[8 + 3 * k], s[9 + 3 * k]) <= s[10 + 3 * k] + p->r_vehicle) return 1;
    return 0;
}

/* get_fake_laser :274-397, literally: obstacles visited in argsort(ref_dis) order, first hit wins */
static void oa_laser(const rlp_ugv_oa_params *p, const double *s, double *laser) {
    double x = s[0], y = s[1], xm = p->map_size[0], ym = p->map_size[1], L = p->laser_dis;
    if (oa_collision(p, s)) {
        for (int i = 0; i < OA_NL; ++i) laser[i] = p->laser_blind;
        return;
    }
    double ref[OA_NOBS];
    int order[OA_NOBS];
    int nob = p->n_obs;
    for (int k = 0; k < nob; ++k) {
        ref[k] = oa_dis(x, y, s[8 + 3 * k], s[9 + 3 * k]);
        order[k] = k;
    }
    for (int k = 1; k < nob; ++k) { /* stable ascending sort */
        int v = order[k], j = k - 1;
        while (j >= 0 && ref[order[j]] > ref[v]) { order[j + 1] = order[j]; --j; }
        order[j + 1] = v;
    }
    double start = s[3] - p->laser_range, stop = s[3] + p->laser_range;
    double step = (stop - start) / (OA_NL - 1); /* np.linspace */
    double th1 = oa_vec_rad(1, 0, xm - x, ym - y);
    double th2 = oa_vec_rad(1, 0, 0 - x, ym - y);
    double th3 = -oa_vec_rad(1, 0, 0 - x, 0 - y);
    double th4 = -oa_vec_rad(1, 0, xm - x, 0 - y);
    for (int i = 0; i < OA_NL; ++i) {
        double ph = i == OA_NL - 1 ? stop : (double)i * step + start;
        if (ph > PI) ph -= 2 * PI;
        if (ph < -PI) ph += 2 * PI;
        double m = tan(ph), b = y - m * x;
        double cosT = fabs(m) / sqrt(1 + m * m), sinT = 1 / sqrt(1 + m * m);
        double tx, ty;
        if (th4 < ph && ph <= th1) {
            tx = xm; ty = m * xm + b;
            if (x + L / sqrt(1 + m * m) < xm) {
                tx = x + L / sqrt(1 + m * m);
                ty = m >= 0 ? y + cosT * L : y - cosT * L;
            }
        } else if (th1 < ph && ph <= th2) {
            if (fabs(m) < 1e8) { tx = (ym - b) / m; ty = ym; } else { tx = x; ty = ym; }
            if (y + fabs(m) * L / sqrt(1 + m * m) < ym) {
                tx = m >= 0 ? x + L * sinT : x - L * sinT;
                ty = y + fabs(m) * L / sqrt(1 + m * m);
            }
        } else if (th3 < ph && ph <= th4) {
            if (fabs(m) < 1e8) { tx = -b / m; ty = 0; } else { tx = x; ty = 0; }
            if (y - fabs(m) * L / sqrt(1 + m * m) > 0) {
                tx = m >= 0 ? x - L * sinT : x + L * sinT;
                ty = y - fabs(m) * L / sqrt(1 + m * m);
            }
        } else {
            tx = 0; ty = b;
            if (x - L / sqrt(1 + m * m) > 0) {
                tx = x - L / sqrt(1 + m * m);
                ty = m >= 0 ? y - cosT * L : y + cosT * L;
            }
        }
        int found = 0;
        for (int kk = 0; kk < nob; ++kk) {
            int k = order[kk];
            double x0 = s[8 + 3 * k], y0 = s[9 + 3 * k], r0 = s[10 + 3 * k];
            if (ref[k] > L + r0) continue;
            if (fabs(m * x0 - y0 + b) / sqrt(1 + m * m) > r0) continue;
            if (oa_vec_rad(tx - x, ty - y, x0 - x, y0 - y) > PI / 2) continue;
            double fx = (x0 + m * y0 - m * b) / (m * m + 1);
            double fy = (m * x0 + m * m * y0 + b) / (m * m + 1);
            double rd = oa_dis(fx, fy, x0, y0);
            double dd = tx - x, sg = dd > 0 ? 1.0 : (dd < 0 ? -1.0 : 0.0);
            double cx = fx - sg * sqrt(r0 * r0 - rd * rd) / sqrt(m * m + 1);
            if (fmin(x, tx) <= cx && cx <= fmax(x, tx)) {
                found = 1;
                double dis = fabs(cx - x) * sqrt(m * m + 1);
                laser[i] = dis < p->laser_blind ? p->laser_blind : dis;
                break;
            }
        }
        if (!found) {
            double dis = oa_dis(x, y, tx, ty);
            if (dis > L) laser[i] = L;
            else if (p->laser_blind < dis && dis <= L) laser[i] = dis;
            else laser[i] = p->laser_blind;
        }
    }
}

static double oa_e(const double *s) { return oa_dis(s[6], s[7], s[0], s[1]); } /* :512-513 */

static double oa_ephi(const double *s) { /* get_e_phi -> cal_vector_rad_oriented */
    double x1 = cos(s[3]), y1 = sin(s[3]), x2 = s[6] - s[0], y2 = s[7] - s[1];
    if (sqrt(x2 * x2 + y2 * y2) < 1e-4 || sqrt(x1 * x1 + y1 * y1) < 1e-4) return 0;
    return atan2(x1 * y2 - y1 * x2, x1 * x2 + y1 * y2);
}

static void oa_obs(const rlp_ugv_oa_params *p, const double *s, float *o) { /* get_state :399-411 */
    double e_max = sqrt(p->map_size[0] * p->map_size[0] + p->map_size[1] * p->map_size[1]) / 2;
    double lz[OA_NL];
    o[0] = (float)((2 / e_max * oa_e(s) - 1) * p->static_gain);
    o[1] = (float)((2 / p->v_max * s[2] - 1) * p->static_gain);
    o[2] = (float)((oa_ephi(s) / p->e_phi_max) * p->static_gain);
    o[3] = (float)((s[4] / p->omega_max) * p->static_gain);
    oa_laser(p, s, lz);
    for (int i = 0; i < OA_NL; ++i) o[4 + i] = (float)((2 * lz[i] / p->laser_dis - 1) * p->static_gain);
}

static void oa_ode(const rlp_ugv_oa_params *p, double al, double aa, const double *x, double *d) {
    d[0] = x[2] * cos(x[3]);
    d[1] = x[2] * sin(x[3]);
    d[2] = al - p->kf * x[2];
    d[3] = x[4];
    d[4] = aa - p->kt * x[4];
}

static void oa_step(const rlp_ugv_oa_params *p, double *s, const float *a, float *obs_cur,
                    float *obs_next, double *reward, int32_t *flag, uint8_t *done) {
    double e_max = sqrt(p->map_size[0] * p->map_size[0] + p->map_size[1] * p->map_size[1]) / 2;
    double c0 = (2 / e_max * oa_e(s) - 1) * p->static_gain; /* current_state[0], [1] (f64) */
    double c1 = (2 / p->v_max * s[2] - 1) * p->static_gain;
    if (obs_cur) oa_obs(p, s, obs_cur);
    double al = (double)a[0], aa = (double)a[1], dt = p->dt; /* rk44 :484-502 */
    double xx[5] = {s[0], s[1], s[2], s[3], s[4]};
    double K1[5], K2[5], K3[5], K4[5], t[5], d[5];
    oa_ode(p, al, aa, xx, d);
    for (int i = 0; i < 5; ++i) { K1[i] = dt * d[i]; t[i] = xx[i] + K1[i] / 2; }
    oa_ode(p, al, aa, t, d);
    for (int i = 0; i < 5; ++i) { K2[i] = dt * d[i]; t[i] = xx[i] + K2[i] / 2; }
    oa_ode(p, al, aa, t, d);
    for (int i = 0; i < 5; ++i) { K3[i] = dt * d[i]; t[i] = xx[i] + K3[i]; }
    oa_ode(p, al, aa, t, d);
    for (int i = 0; i < 5; ++i) { K4[i] = dt * d[i]; xx[i] = xx[i] + (K1[i] + 2 * K2[i] + 2 * K3[i] + K4[i]) / 6; }
    if (p->shaped) { /* demo copy rk44 :496-500 tests the pre-step vel */
        if (s[2] < 0.) { s[3] = xx[3]; s[4] = xx[4]; s[2] = 0.; }
        else { for (int i = 0; i < 5; ++i) s[i] = xx[i]; }
    } else {
        for (int i = 0; i < 5; ++i) s[i] = xx[i];
        if (s[2] < 0.) s[2] = 0.;
    }
    s[5] = s[5] + dt;
    if (s[3] > PI) s[3] -= 2 * PI;
    if (s[3] < -PI) s[3] += 2 * PI;
    double e = oa_e(s), eph = oa_ephi(s);
    int f = 0; /* is_Terminal :433-450 */
    if (s[0] > p->map_size[0] || s[0] < 0 || s[1] > p->map_size[1] || s[1] < 0) f = 1;
    if (s[5] > p->time_max) f = 2;
    int success = fabs(e) <= 0.05 && (p->shaped ? 1 : fabs(s[4]) < 0.01) && fabs(s[2]) < 0.01;
    if (success) f = 3;
    if (oa_collision(p, s)) f = 4;
    oa_obs(p, s, obs_next);
    *flag = f;
    *done = f != 0;
    if (p->shaped) { /* demo copy get_reward :449-473 */
        double n0 = (2 / e_max * e - 1) * p->static_gain, n1 = (2 / p->v_max * s[2] - 1) * p->static_gain;
        double r1 = -1 - fabs(s[4]) * 0.1, r2, r3, r4;
        if (c0 > n0 + 1e-3) r2 = 5; else if (1e-3 + c0 < n0) r2 = -5; else r2 = 0;
        if (fabs(c1) > fabs(n1) + 1e-2) r3 = 2; else if (1e-2 + fabs(c1) < fabs(n1)) r3 = -2; else r3 = 0;
        if (success) r4 = 500; else if (f == 4) r4 = -300; else r4 = 0;
        *reward = r1 + r2 + r3 + r4;
        return;
    }
    double u_pos = -fabs(e) * p->Q_pos; /* get_reward :452-469 */
    double u_vel = -fabs(s[2]) * p->Q_vel;
    double u_phi = e > 0.1 ? -fabs(eph) * p->Q_phi : 0.0;
    double u_om = -fabs(s[4]) * p->Q_omega;
    double u_psi = 0.;
    if (f == 1) u_psi = (p->time_max - s[5]) / p->dt * (u_pos + u_vel + u_phi + u_om);
    *reward = u_pos + u_vel + u_phi + u_om + u_psi;
}

/* reset(random=True) :520-557 + map.py:66-174 generate_circle_obs_training: sequential rejection
 * sampling. Each draw is Philox-keyed by what it is: start 0x40000000, target try t 0x41000000 + t,
 * obstacle k try t 0x42000000 / 0x42800000 + (k << 16) + t, heading 0x43000000. */
static void oa_draw_point(const rlp_ugv_oa_params *p, uint64_t seed, uint64_t counter,
                          uint64_t id, uint32_t tag, double *x, double *y) { /* map.py:66-74 */
    double u[2], mg = p->st_margin;
    philox_u01_f64x2(seed, counter, id, tag, u);
    *x = mg + ((p->map_size[0] - mg) - mg) * u[0];
    *y = mg + ((p->map_size[1] - mg) - mg) * u[1];
}

static void oa_reset(const rlp_ugv_oa_params *p, double *s, uint64_t seed, uint64_t counter,
                     uint64_t env_id) {
    double sx, sy, tx, ty, u[2], v[2];
    oa_draw_point(p, seed, counter, env_id, 0x40000000u, &sx, &sy);
    tx = sx; ty = sy;
    for (int t = 0; t < p->max_tries && oa_dis(tx, ty, sx, sy) < p->safety_dis_st; ++t)
        oa_draw_point(p, seed, counter, env_id, 0x41000000u + (uint32_t)t, &tx, &ty);
    for (int k = 0; k < OA_NOBS; ++k) {
        double cx = -1000.0 - 10.0 * k, cy = -1000.0, r = p->r_min; /* parked */
        for (int t = 0; k < p->n_obs && t < p->max_tries; ++t) {
            uint32_t kt = ((uint32_t)k << 16) + (uint32_t)t;
            philox_u01_f64x2(seed, counter, env_id, 0x42000000u + kt, u);
            philox_u01_f64x2(seed, counter, env_id, 0x42800000u + kt, v);
            double ccx = 0 + (p->map_size[0] - 0) * u[0], ccy = 0 + (p->map_size[1] - 0) * u[1];
            double rr = p->r_min + (p->r_max - p->r_min) * v[0];
            int ok = oa_dis(sx, sy, ccx, ccy) > rr + p->safety_dis_st &&
                     oa_dis(tx, ty, ccx, ccy) > rr + p->safety_dis_st;
            for (int j = 0; j < k && ok; ++j) /* __is_new_obs_in_obs: r_existing + r_new + safety */
                if (oa_dis(s[8 + 3 * j], s[9 + 3 * j], ccx, ccy) <= s[10 + 3 * j] + rr + p->safety_dis_obs) ok = 0;
            if (ok) { cx = ccx; cy = ccy; r = rr; break; }
        }
        s[8 + 3 * k] = cx; s[9 + 3 * k] = cy; s[10 + 3 * k] = r;
    }
    philox_u01_f64x2(seed, counter, env_id, 0x43000000u, u);
    s[0] = sx; s[1] = sy; s[2] = 0.; s[3] = -PI + (PI - -PI) * u[0]; s[4] = 0.; s[5] = 0.;
    s[6] = tx; s[7] = ty;
}

/* ------------------------------------------------------------------------------------------ */
/* Generic entry points (kind dispatch), SoA state [D][n]                                      */
/* ------------------------------------------------------------------------------------------ */
int oracle_env_dims(int kind, int *D, int *S, int *A) {
    switch (kind) {
    case RLP_ENV_CARTPOLE: *D = RLP_CARTPOLE_D; *S = 4; *A = 1; return 0;
    case RLP_ENV_CARTPOLE_ANGLEONLY: *D = RLP_ANGLEONLY_D; *S = 2; *A = 1; return 0;
    case RLP_ENV_SOI: *D = RLP_SOI_D; *S = 4; *A = 2; return 0;
    case RLP_ENV_UGV_FORWARD:
    case RLP_ENV_UGV_BIDIRECTIONAL: *D = RLP_UGV_D; *S = 4; *A = 2; return 0;
    case RLP_ENV_UAV_HOVER_OUTER_LOOP: *D = RLP_UAV_D; *S = 6; *A = 3; return 0;
    case RLP_ENV_UGV_OBSTACLE_AVOIDANCE: *D = RLP_UGVOA_D; *S = 4 + OA_NL; *A = 2; return 0;
    }
    return -1;
}

static void gather(const double *state, int D, int n, int i, double *s) {
    for (int d = 0; d < D; ++d) s[d] = state[(size_t)d * n + i];
}
static void scatter(double *state, int D, int n, int i, const double *s) {
    for (int d = 0; d < D; ++d) state[(size_t)d * n + i] = s[d];
}

static void env_step1(int kind, const void *params, double *s, const float *a, float *oc,
                      float *on, double *r, int32_t *f, uint8_t *dn) {
    switch (kind) {
    case RLP_ENV_CARTPOLE: cp_step((const rlp_cartpole_params *)params, s, a[0], oc, on, r, f, dn); break;
    case RLP_ENV_CARTPOLE_ANGLEONLY: ao_step((const rlp_angleonly_params *)params, s, a[0], oc, on, r, f, dn); break;
    case RLP_ENV_SOI: soi_step((const rlp_soi_params *)params, s, a, oc, on, r, f, dn); break;
    case RLP_ENV_UGV_FORWARD: ugv_step((const rlp_ugv_params *)params, 0, s, a, oc, on, r, f, dn); break;
    case RLP_ENV_UGV_BIDIRECTIONAL: ugv_step((const rlp_ugv_params *)params, 1, s, a, oc, on, r, f, dn); break;
    case RLP_ENV_UAV_HOVER_OUTER_LOOP: uav_step((const rlp_uav_hover_params *)params, s, a, oc, on, r, f, dn); break;
    case RLP_ENV_UGV_OBSTACLE_AVOIDANCE: oa_step((const rlp_ugv_oa_params *)params, s, a, oc, on, r, f, dn); break;
    }
}

static void env_obs1(int kind, const void *params, const double *s, float *o) {
    switch (kind) {
    case RLP_ENV_CARTPOLE: cp_obs((const rlp_cartpole_params *)params, s, o); break;
    case RLP_ENV_CARTPOLE_ANGLEONLY: ao_obs((const rlp_angleonly_params *)params, s, o); break;
    case RLP_ENV_SOI: soi_obs((const rlp_soi_params *)params, s, o); break;
    case RLP_ENV_UGV_FORWARD: ugv_obs((const rlp_ugv_params *)params, 0, s, o); break;
    case RLP_ENV_UGV_BIDIRECTIONAL: ugv_obs((const rlp_ugv_params *)params, 1, s, o); break;
    case RLP_ENV_UAV_HOVER_OUTER_LOOP: uav_obs((const rlp_uav_hover_params *)params, s, o); break;
    case RLP_ENV_UGV_OBSTACLE_AVOIDANCE: oa_obs((const rlp_ugv_oa_params *)params, s, o); break;
    }
}

int oracle_env_step(int kind, const void *params, double *state, int n, const float *action,
                    float *obs_cur, float *obs_next, double *reward, int32_t *flag, uint8_t *done) {
    int D, S, A;
    if (oracle_env_dims(kind, &D, &S, &A)) return -1;
    /* independent envs: OpenMP over them (oracle_set_threads), each env's arithmetic unchanged */
#pragma omp parallel for schedule(static) if (n > 256)
    for (int i = 0; i < n; ++i) {
        double s[64];
        gather(state, D, n, i, s);
        env_step1(kind, params, s, action + (size_t)i * A, obs_cur ? obs_cur + (size_t)i * S : NULL,
                  obs_next + (size_t)i * S, reward + i, flag + i, done + i);
        scatter(state, D, n, i, s);
    }
    return 0;
}

int oracle_env_observe(int kind, const void *params, const double *state, int n, float *obs) {
    int D, S, A;
    if (oracle_env_dims(kind, &D, &S, &A)) return -1;
    double s[64];
    for (int i = 0; i < n; ++i) {
        gather(state, D, n, i, s);
        env_obs1(kind, params, s, obs + (size_t)i * S);
    }
    return 0;
}

/* reset law of each kind with the Philox stream (tag 0x200+j), keeping carried hidden state */
static void env_reset1(int kind, const void *params, double *s, uint64_t seed, uint64_t counter,
                       uint64_t env_id) {
    double u[2];
    switch (kind) {
    case RLP_ENV_CARTPOLE: { /* CartPole.py:272-282 */
        const rlp_cartpole_params *p = (const rlp_cartpole_params *)params;
        philox_u01_f64x2(seed, counter, env_id, 0x200u, u);
        s[0] = p->reset_theta_lo + (p->reset_theta_hi - p->reset_theta_lo) * u[0];
        s[1] = 0.;
        s[2] = p->reset_x_lo + (p->reset_x_hi - p->reset_x_lo) * u[1];
        s[3] = 0.;
        s[4] = 0.;
        break;
    }
    case RLP_ENV_CARTPOLE_ANGLEONLY: { /* cartpole_angleonly.py:250-262 */
        const rlp_angleonly_params *p = (const rlp_angleonly_params *)params;
        philox_u01_f64x2(seed, counter, env_id, 0x200u, u);
        s[0] = p->reset_theta_lo + (p->reset_theta_hi - p->reset_theta_lo) * u[0];
        s[1] = 0.; s[2] = 0.; s[3] = 0.; s[4] = 0.;
        break;
    }
    case RLP_ENV_SOI: { /* SecondOrderIntegration.py:329-339 */
        const rlp_soi_params *p = (const rlp_soi_params *)params;
        philox_u01_f64x2(seed, counter, env_id, 0x200u, u);
        double lo = 0 + p->reset_margin;
        s[0] = lo + ((p->map_size[0] - p->reset_margin) - lo) * u[0];
        s[1] = lo + ((p->map_size[1] - p->reset_margin) - lo) * u[1];
        s[2] = 0.; s[3] = 0.; s[4] = 0.;
        s[5] = p->map_size[0] / 2; s[6] = p->map_size[1] / 2;
        break;
    }
    case RLP_ENV_UGV_FORWARD:
    case RLP_ENV_UGV_BIDIRECTIONAL: { /* UGVForward.py:335-350 */
        const rlp_ugv_params *p = (const rlp_ugv_params *)params;
        double u2[2];
        philox_u01_f64x2(seed, counter, env_id, 0x200u, u);
        philox_u01_f64x2(seed, counter, env_id, 0x201u, u2);
        double d0 = p->reset_margin;
        s[0] = d0 + ((p->map_size[0] - d0) - d0) * u[0];
        s[1] = d0 + ((p->map_size[1] - d0) - d0) * u[1];
        s[3] = -PI + (PI - -PI) * u2[0];
        s[2] = 0.; s[4] = 0.; s[5] = 0.;
        s[6] = p->map_size[0] / 2; s[7] = p->map_size[1] / 2;
        break;
    }
    case RLP_ENV_UAV_HOVER_OUTER_LOOP: { /* UavHoverOuterLoop.py:152-214 */
        const rlp_uav_hover_params *p = (const rlp_uav_hover_params *)params;
        double u2[2];
        philox_u01_f64x2(seed, counter, env_id, 0x200u, u);
        philox_u01_f64x2(seed, counter, env_id, 0x201u, u2);
        for (int i = 0; i < 3; ++i) {
            s[U_X + i] = p->pos0[i]; s[U_VX + i] = p->vel0[i];
            s[U_PHI + i] = p->angle0[i]; s[U_P + i] = p->pqr0[i];
        }
        s[U_T] = 0.;
        double uu[3] = {u[0], u[1], u2[0]};
        for (int i = 0; i < 3; ++i) {
            double lo = p->pos_zone[i][0] + p->target_offset, hi = p->pos_zone[i][1] - p->target_offset;
            s[U_REF + i] = lo + (hi - lo) * uu[i];
        }
        /* s1 and att_ref are NOT reset (carried over, as in the reference) */
        break;
    }
    case RLP_ENV_UGV_OBSTACLE_AVOIDANCE:
        oa_reset((const rlp_ugv_oa_params *)params, s, seed, counter, env_id);
        break;
    }
}

int oracle_env_reset(int kind, const void *params, double *state, int n, const uint8_t *mask,
                     const double *init_state, uint64_t seed, uint64_t counter, uint64_t env_id0) {
    int D, S, A;
    if (oracle_env_dims(kind, &D, &S, &A)) return -1;
    double s[64];
    for (int i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        if (init_state) {
            for (int d = 0; d < D; ++d) state[(size_t)d * n + i] = init_state[(size_t)d * n + i];
        } else {
            gather(state, D, n, i, s);
            env_reset1(kind, params, s, seed, counter, env_id0 + (uint64_t)i);
            scatter(state, D, n, i, s);
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* MLP forward (torch nn.Linear stacks), double accumulation, fp32 in/out                     */
/* ------------------------------------------------------------------------------------------ */
int oracle_mlp_forward(const rlp_mlp_desc *desc, const float *params, const float *x, float *y,
                       int n) {
    int maxw = 0;
    for (int l = 0; l <= desc->n_layers; ++l) maxw = desc->dims[l] > maxw ? desc->dims[l] : maxw;
#pragma omp parallel if (n > 64)
    {
    double *a = (double *)malloc(sizeof(double) * maxw), *b = (double *)malloc(sizeof(double) * maxw);
#pragma omp for schedule(static)
    for (int i = 0; i < n; ++i) {
        for (int k = 0; k < desc->dims[0]; ++k) a[k] = x[(size_t)i * desc->dims[0] + k];
        const float *pw = params;
        for (int l = 0; l < desc->n_layers; ++l) {
            int in = desc->dims[l], out = desc->dims[l + 1];
            const float *W = pw, *bb = pw + (size_t)in * out;
            for (int j = 0; j < out; ++j) {
                double acc = 0;
                for (int k = 0; k < in; ++k) acc += (double)W[(size_t)j * in + k] * a[k];
                acc += bb[j];
                float v = (float)acc; /* torch materialises every layer in fp32 */
                if (desc->act[l] == RLP_ACT_TANH) v = (float)tanh((double)v);
                else if (desc->act[l] == RLP_ACT_RELU) v = v > 0 ? v : 0;
                b[j] = v;
            }
            pw += (size_t)in * out + out;
            double *t = a; a = b; b = t;
        }
        for (int j = 0; j < desc->dims[desc->n_layers]; ++j)
            y[(size_t)i * desc->dims[desc->n_layers] + j] = (float)a[j];
    }
    free(a);
    free(b);
    }
    return 0;
}

/* Normal(mean, std).log_prob(a) of torch.distributions (fp32 expression order):
 * -((a - mean)^2) / (2 var) - log(std) - log(sqrt(2 pi)) */
static float normal_logp(float a, float mean, float std) {
    float var = std * std;
    float d = a - mean;
    return -(d * d) / (2.0f * var) - logf(std) - 0.91893853320467274178f;
}

int oracle_policy_sample(const float *mean, int n, int A, const float *std, const float *a_min,
                         const float *a_max, const float *noise, uint64_t seed, uint64_t counter,
                         uint64_t env_id0, float *action, float *logp) {
    float eps[8];
    for (int i = 0; i < n; ++i) {
        if (noise) {
            for (int j = 0; j < A; ++j) eps[j] = noise[(size_t)i * A + j];
        } else {
            oracle_philox_normal_f32(seed, counter, env_id0 + (uint64_t)i, A, eps);
        }
        for (int j = 0; j < A; ++j) {
            float m = mean[(size_t)i * A + j];
            float a = m + std[j] * eps[j];
            a = fmaxf(fminf(a, a_max[j]), a_min[j]);
            action[(size_t)i * A + j] = a;
            logp[(size_t)i * A + j] = normal_logp(a, m, std[j]);
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Learn-side scans                                                                            */
/* ------------------------------------------------------------------------------------------ */
/* GAE, Proximal_Policy_Optimization2.py:91-98 in NumPy-2 fp32 order */
int oracle_gae(const float *r, const float *v, const float *vn, const uint8_t *done,
               const uint8_t *success, double gamma, double lambda, int T, int n, float *adv,
               float *vt) {
    float g32 = (float)gamma;
    float c = (float)(gamma * lambda);
    for (int i = 0; i < n; ++i) {
        float gae = 0.f;
        for (int t = T - 1; t >= 0; --t) {
            size_t k = (size_t)t * n + i;
            float one_s = 1.0f - (float)success[k];
            float delta = r[k] + (g32 * one_s) * vn[k];
            delta = delta - v[k];
            float tt = c * gae;
            tt = tt * (1.0f - (float)done[k]);
            gae = delta + tt;
            adv[k] = gae;
            vt[k] = gae + v[k];
        }
    }
    return 0;
}

/* Normalization(shape=1) — utils/classes.py:626-656; batched merge per time step (see rlp.h) */
int oracle_reward_norm(const float *rin, int T, int n, double *rms, float *rout) {
    for (int t = 0; t < T; ++t) {
        const float *x = rin + (size_t)t * n;
        double cnt = rms[0], mean = rms[1], S = rms[2], sd = rms[3];
        if (n == 1) {
            double xv = (double)x[0];
            cnt += 1;
            if (cnt == 1) { mean = xv; sd = xv; }
            else {
                double old = mean;
                mean = old + (xv - old) / cnt;
                S = S + (xv - old) * (xv - mean);
                sd = sqrt(S / cnt);
            }
        } else {
            double mb = 0;
            for (int i = 0; i < n; ++i) mb += (double)x[i];
            mb /= n;
            double Sb = 0;
            for (int i = 0; i < n; ++i) { double d = (double)x[i] - mb; Sb += d * d; }
            if (cnt == 0) { cnt = n; mean = mb; S = Sb; }
            else {
                double nn = cnt + n;
                double dl = mb - mean;
                mean = mean + dl * ((double)n / nn);
                S = S + Sb + dl * dl * (cnt * (double)n / nn);
                cnt = nn;
            }
            sd = sqrt(S / cnt);
        }
        rms[0] = cnt; rms[1] = mean; rms[2] = S; rms[3] = sd;
        for (int i = 0; i < n; ++i)
            rout[(size_t)t * n + i] = (float)(((double)x[i] - mean) / (sd + 1e-8));
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Whole rollout segment (the reference driver loop, batched): used as the CPU baseline and as */
/* the closed-loop parity reference of rlp_rollout.                                            */
/* ------------------------------------------------------------------------------------------ */
/* The batched driver loop (demonstration/PPO2/PPO2-4-CartPole/train.py:184-217 with the reset of
 * :186-190 and the success rules of rlp.h) for n independent envs, one env after another.
 *
 * forced_action [T][n][A] (nullable): teacher forcing. The env is stepped with the given actions
 * (e.g. the ones a GPU rollout stored) while the buffers still record the oracle's own policy
 * output (mean + std * Philox noise, clamped) and critic value for the oracle's own observations,
 * so a GPU run can be checked step by step without the closed loop amplifying the ~1e-7
 * difference between its f32 MLP and this double-accumulated one. actor == NULL (only with
 * forced_action) skips the nets altogether: physics, rewards, flags and resets only (action,
 * logp, value and value_next are then left untouched).
 *
 * Envs are independent: with OpenMP the env loop runs on all host threads (same results). */
int oracle_rollout_forced(int kind, const void *env_params, double *state, uint8_t *need_reset,
                          const rlp_mlp_desc *ad, const float *actor, const rlp_mlp_desc *cd,
                          const float *critic, const rlp_rollout_cfg *cfg,
                          const rlp_rollout_bufs *b, const float *forced_action) {
    int D, S, A;
    if (oracle_env_dims(kind, &D, &S, &A)) return -1;
    if (!actor && !forced_action) return -1;
    int n = cfg->n;
    float gain[4], off[4];
    for (int j = 0; j < A; ++j) {
        off[j] = (cfg->a_min[j] + cfg->a_max[j]) / 2.0f;
        gain[j] = cfg->a_max[j] - off[j];
    }
    const int nets = actor != NULL;
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; ++i) {
        double s[64];
        float o[64], on[64], mean[8], eps[8], act[8], lp[8], v = 0.f;
        gather(state, D, n, i, s);
        uint64_t eid = cfg->env_id0 + (uint64_t)i;
        for (int t = 0; t < cfg->T; ++t) {
            uint64_t g = cfg->step0 + (uint64_t)t;
            size_t k = (size_t)t * n + i;
            if (need_reset[i]) {
                env_reset1(kind, env_params, s, cfg->seed, g, eid);
                need_reset[i] = 0;
            }
            env_obs1(kind, env_params, s, o);
            if (nets) {
                oracle_mlp_forward(ad, actor, o, mean, 1);
                for (int j = 0; j < A; ++j) mean[j] = mean[j] * gain[j] + off[j];
                oracle_mlp_forward(cd, critic, o, &v, 1);
                oracle_philox_normal_f32(cfg->seed, g, eid, A, eps);
                for (int j = 0; j < A; ++j) {
                    float a = mean[j] + cfg->std[j] * eps[j];
                    a = fmaxf(fminf(a, cfg->a_max[j]), cfg->a_min[j]);
                    act[j] = a;
                    lp[j] = normal_logp(a, mean[j], cfg->std[j]);
                }
            }
            double r;
            int32_t f;
            uint8_t dn;
            env_step1(kind, env_params, s, forced_action ? forced_action + k * A : act, NULL, on,
                      &r, &f, &dn);
            int su;
            switch (cfg->success_rule) {
            case RLP_SUCCESS_FLAG_NE: su = f != cfg->success_flag; break;
            case RLP_SUCCESS_FLAG_EQ: su = f == cfg->success_flag; break;
            default: su = dn && f != cfg->success_flag; break;
            }
            if (b) {
                for (int q = 0; q < S; ++q) {
                    b->obs[k * S + q] = o[q];
                    b->obs_next[k * S + q] = on[q];
                }
                if (nets) {
                    for (int j = 0; j < A; ++j) {
                        b->action[k * A + j] = act[j];
                        b->logp[k * A + j] = lp[j];
                    }
                    b->value[k] = v;
                    if (t > 0 && !b->done[k - n]) b->value_next[k - n] = v;
                }
                b->reward[k] = (float)r;
                b->done[k] = dn;
                b->success[k] = (uint8_t)su;
                b->flag[k] = (int8_t)f;
            }
            if (dn) need_reset[i] = 1;
        }
        if (b && nets && !need_reset[i]) {
            env_obs1(kind, env_params, s, o);
            oracle_mlp_forward(cd, critic, o, &v, 1);
            b->value_next[(size_t)(cfg->T - 1) * n + i] = v;
        }
        scatter(state, D, n, i, s);
    }
    return 0;
}

int oracle_rollout(int kind, const void *env_params, double *state, uint8_t *need_reset,
                   const rlp_mlp_desc *ad, const float *actor, const rlp_mlp_desc *cd,
                   const float *critic, const rlp_rollout_cfg *cfg, const rlp_rollout_bufs *b) {
    return oracle_rollout_forced(kind, env_params, state, need_reset, ad, actor, cd, critic, cfg,
                                 b, NULL);
}

/* Host threads for the env / row loops (bench.py's cpu_baseline times 1 and all cores). */
int oracle_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}
