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

// the head of get_state (e, vel, e_phi, omega) of a pose
__device__ __forceinline__ void oa_head(const OA::P &p, const double *s, float *row) {
    float h[4];
    OA::obs_head(p, s, OA::get_e(s), OA::e_phi(s), h);
#pragma unroll
    for (int j = 0; j < 4; ++j) row[j] = h[j];
}

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

// the same setup of ONE env by a whole wave (wave-uniform call, every lane the same pose s): lane
// k < n_obs obstacle k's distance and collision test (collision_at's any() as a ballot), lanes
// 0..3 the four corner angles (one acos each), lane 4 the beam angles; lane 5 writes get_state's
// head into head_row (nullable). The caller orders the LDS writes before any read (wave barrier).
__device__ __forceinline__ void oa_setup_wave(const OA::P &p, OaEnvLds &L, const double *s,
                                              float *head_row, float *head_row2 = nullptr) {
    const int lane = threadIdx.x & 63;
    const double x = s[OA::X], y = s[OA::Y];
    bool hit = false;
    if (lane < p.n_obs) {
        const double dx = x - L.ob[lane].x0, dy = y - L.ob[lane].y0;
        const double d = sqrt(dx * dx + dy * dy);
        L.ob[lane].ref = d;
        hit = d <= L.ob[lane].r0 + p.r_vehicle;
    }
    const bool coll = __ballot(hit) != 0;
    if (lane < 4) {  // pose(): th1 (xm, ym), th2 (0, ym), th3 -(0, 0), th4 -(xm, 0) corners
        const double cx = (lane == 0 || lane == 3) ? p.map_size[0] - x : 0 - x;
        const double cy = (lane == 0 || lane == 1) ? p.map_size[1] - y : 0 - y;
        const double v = OA::vec_rad(1, 0, cx, cy);
        if (lane == 0) L.q.th1 = v;
        else if (lane == 1) L.q.th2 = v;
        else if (lane == 2) L.q.th3 = -v;
        else L.q.th4 = -v;
    } else if (lane == 4) {
        L.q.x = x;
        L.q.y = y;
        L.q.start = s[OA::PHI] - p.laser_range;
        L.q.stop = s[OA::PHI] + p.laser_range;
        L.q.step = (L.q.stop - L.q.start) / (OA::NL - 1);
        L.coll = coll;
    } else if (lane == 5 && head_row) {
        oa_head(p, s, head_row);
        if (head_row2)
            for (int j = 0; j < 4; ++j) head_row2[j] = head_row[j];
    }
}

// beam i of an env set up in L (get_state's normalised value)
__device__ __forceinline__ float oa_beam(const OA::P &p, const OaEnvLds &L, int i) {
    if (L.coll) return OA::beam_obs(p, p.laser_blind);
    const OA::Pose q = L.q;
    return OA::beam_obs(p, OA::beam<true>(p, q, i, [&](int k, double &x0, double &y0, double &r0,
                                                       double &rf) {
        const OaObstacle o = L.ob[k];
        x0 = o.x0; y0 = o.y0; r0 = o.r0; rf = o.ref;
    }));
}

// reset(random=True) of env i by ONE wave (all 64 lanes, wave-uniform call): each round, lane l
// tests try (round * 64 + l) of the target / of obstacle k, and the lowest legal try wins — the
// sequential sampler's result (Env<7>::reset) at ~1 round per draw instead of the wave waiting on
// its unluckiest lane. Writes every state component of env i; with obs_row != nullptr also the new
// pose's observation (head + the 37 beams, one per lane). obl (NOBS * 3 doubles) and L: this
// wave's LDS scratch.
__device__ __forceinline__ void oa_reset_wave(const OA::P &p, double *state, int n, size_t i,
                                              uint64_t seed, uint64_t counter, uint64_t id,
                                              float *obs_row, double *obl, OaEnvLds &L,
                                              float *obs_row2 = nullptr) {
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
    // the first round's draw of obstacle k + 1 (try = lane) does not depend on where obstacle k
    // lands: it is drawn before obstacle k's legality checks, so the chain per obstacle is the
    // checks and the ballot, not the two Philox blocks (later rounds, rare, draw in turn)
    double nx = 0, ny = 0, nr = 0;
    if (p.n_obs > 0 && lane < p.max_tries) OA::draw_obstacle(p, seed, counter, id, 0, lane, nx, ny, nr);
    for (int k = 0; k < OA::NOBS; ++k) {
        double cx = OA::parked_x(k), cy = OA::kParkedY, r = p.r_min;
        const double fx = nx, fy = ny, fr = nr;  // round 0 of obstacle k
        if (k + 1 < p.n_obs && lane < p.max_tries)
            OA::draw_obstacle(p, seed, counter, id, k + 1, lane, nx, ny, nr);
        for (int t0 = 0; k < p.n_obs && t0 < p.max_tries; t0 += 64) {
            const int t = t0 + lane;
            double ccx = fx, ccy = fy, rr = fr;
            bool ok = false;
            if (t < p.max_tries) {
                if (t0 > 0) OA::draw_obstacle(p, seed, counter, id, k, t, ccx, ccy, rr);
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
    if (lane < p.n_obs) {  // the per-pose setup of the new pose, over the wave's lanes
        L.ob[lane].x0 = obl[3 * lane];
        L.ob[lane].y0 = obl[3 * lane + 1];
        L.ob[lane].r0 = obl[3 * lane + 2];
    }
    oa_setup_wave(p, L, head, obs_row, obs_row2);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < OA::NL) {  // one beam per lane
        const float v = oa_beam(p, L, lane);
        obs_row[4 + lane] = v;
        if (obs_row2) obs_row2[4 + lane] = v;
    }
}

}  // namespace rlp
