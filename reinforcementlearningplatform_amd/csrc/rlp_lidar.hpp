// rlp_lidar.hpp — UGVForwardObstacleAvoidance pieces shared by the env-step kernels
// (rlp_lidar.hip) and the fused rollout step (rlp_rollout.hip): the per-env LDS record of a scan
// (obstacles, pose geometry, collision), its setup by the env's lane, the beam scan with one
// (env, beam) pair per lane, and reset(random=True) by one wave per env.
// Reference: environment/UGVForwardObstacleAvoidance/UGVForwardObstacleAvoidance.py get_fake_laser
// :274-397, collision_check :261-272, reset :520-557, map.py:66-174.
#pragma once
#include "rlp_envs.hpp"

namespace rlp {

using OA = Env<RLP_ENV_UGV_OBSTACLE_AVOIDANCE>;

struct alignas(16) OaObstacle {
    double x0, y0, r0, ref;  // ref = distance from the pose being scanned
};

// one env's scan in LDS
struct OaEnvLds {
    OaObstacle ob[OA::NOBS];
    OA::Pose q;
    int coll;
};

// per-pose setup by the env's lane: obstacle distances, collision and the beam geometry
__device__ __forceinline__ void oa_setup(const OA::P &p, OaEnvLds &L, const double *s) {
    const double x = s[OA::X], y = s[OA::Y];
    for (int k = 0; k < p.n_obs; ++k) {
        const double dx = x - L.ob[k].x0, dy = y - L.ob[k].y0;
        L.ob[k].ref = sqrt(dx * dx + dy * dy);
    }
    L.coll = OA::collision_at(p, x, y, [&](int k, double &x0, double &y0, double &r0) {
        x0 = L.ob[k].x0; y0 = L.ob[k].y0; r0 = L.ob[k].r0;
    });
    L.q = OA::pose(p, x, y, s[OA::PHI]);
}

// beam i of an env set up in L (get_state's normalised value)
__device__ __forceinline__ float oa_beam(const OA::P &p, const OaEnvLds &L, int i) {
    if (L.coll) return OA::beam_obs(p, p.laser_blind);
    const OA::Pose q = L.q;
    return OA::beam_obs(p, OA::beam(p, q, i, [&](int k, double &x0, double &y0, double &r0,
                                                 double &rf) {
        const OaObstacle o = L.ob[k];
        x0 = o.x0; y0 = o.y0; r0 = o.r0; rf = o.ref;
    }));
}

// the head of get_state (e, vel, e_phi, omega) of a pose
__device__ __forceinline__ void oa_head(const OA::P &p, const double *s, float *row) {
    float h[4];
    OA::obs_head(p, s, OA::get_e(s), OA::e_phi(s), h);
#pragma unroll
    for (int j = 0; j < 4; ++j) row[j] = h[j];
}

// reset(random=True) of env i by ONE wave (all 64 lanes, wave-uniform call): each round, lane l
// tests try (round * 64 + l) of the target / of obstacle k, and the lowest legal try wins — the
// sequential sampler's result (Env<7>::reset) at ~1 round per draw instead of the wave waiting on
// its unluckiest lane. Writes every state component of env i; with obs_row != nullptr also the new
// pose's observation (head + the 37 beams, one per lane). obl (NOBS * 3 doubles) and L: this
// wave's LDS scratch.
__device__ __forceinline__ void oa_reset_wave(const OA::P &p, double *state, int n, size_t i,
                                              uint64_t seed, uint64_t counter, uint64_t id,
                                              float *obs_row, double *obl, OaEnvLds &L) {
    const int lane = threadIdx.x & 63;
    double sx, sy;
    OA::draw_point(p, seed, counter, id, OA::kTagStart, sx, sy);
    double tx = sx, ty = sy;
    if (!(0.0 >= p.safety_dis_st)) {  // terminal = start fails the distance test: redraw
        for (int t0 = 0; t0 < p.max_tries; t0 += 64) {
            const int t = t0 + lane;
            double cx = 0, cy = 0;
            bool ok = false;
            if (t < p.max_tries) {
                OA::draw_point(p, seed, counter, id, OA::kTagTarget + (uint32_t)t, cx, cy);
                const double dx = cx - sx, dy = cy - sy;
                ok = sqrt(dx * dx + dy * dy) >= p.safety_dis_st;
            }
            const uint64_t b = __ballot(ok);
            const bool last = t0 + 64 >= p.max_tries;
            if (b || last) {  // first legal try, else the last try drawn
                const int src = b ? __ffsll((unsigned long long)b) - 1 : (p.max_tries - 1 - t0);
                tx = __shfl(cx, src);
                ty = __shfl(cy, src);
                break;
            }
        }
    }
    for (int k = 0; k < OA::NOBS; ++k) {
        double cx = OA::parked_x(k), cy = OA::kParkedY, r = p.r_min;
        for (int t0 = 0; k < p.n_obs && t0 < p.max_tries; t0 += 64) {
            const int t = t0 + lane;
            double ccx = 0, ccy = 0, rr = 0;
            bool ok = false;
            if (t < p.max_tries) {
                OA::draw_obstacle(p, seed, counter, id, k, t, ccx, ccy, rr);
                ok = OA::legal(p, sx, sy, tx, ty, ccx, ccy, rr, k,
                               [&](int j, double &x0, double &y0, double &r0) {
                                   x0 = obl[3 * j]; y0 = obl[3 * j + 1]; r0 = obl[3 * j + 2];
                               });
            }
            const uint64_t b = __ballot(ok);
            if (b) {
                const int src = __ffsll((unsigned long long)b) - 1;
                cx = __shfl(ccx, src);
                cy = __shfl(ccy, src);
                r = __shfl(rr, src);
                break;
            }
        }
        if (lane == 0) {
            obl[3 * k] = cx;
            obl[3 * k + 1] = cy;
            obl[3 * k + 2] = r;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    double u[2];
    philox_u01_f64x2(seed, counter, id, OA::kTagPhi, u);
    const double head[OA::DW] = {sx, sy, 0., -kPi + (kPi - -kPi) * u[0], 0., 0., tx, ty};
    if (lane < OA::DW) {
        double v = head[0];
#pragma unroll
        for (int d = 1; d < OA::DW; ++d) v = lane == d ? head[d] : v;
        state[(size_t)lane * n + i] = v;
    }
    if (lane < OA::NOBS * 3) state[(size_t)(OA::OB + lane) * n + i] = obl[lane];
    if (!obs_row) return;
    if (lane == 0) {  // the per-pose setup of the new pose, for this wave's env
        for (int k = 0; k < p.n_obs; ++k) {
            L.ob[k].x0 = obl[3 * k];
            L.ob[k].y0 = obl[3 * k + 1];
            L.ob[k].r0 = obl[3 * k + 2];
        }
        oa_setup(p, L, head);
        oa_head(p, head, obs_row);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < OA::NL) obs_row[4 + lane] = oa_beam(p, L, lane);  // one beam per lane
}

}  // namespace rlp
