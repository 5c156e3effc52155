// k_nn.hip — the correspondence search of one ICP iteration, batched over every active pair.
//
//   SE(3) phase: exact 1-NN of each source SE(3) element under the weighted SE(3) metric
//                (12-D L2), update_correspondences_raw_flann_SE3 ISR.cpp:444-470;
//   R3 phase:    exact 3-D 1-NN, update_correspondences_kd_tree_XYZ ISR.cpp:402-416.
//
// One wavefront = one leaf (<= 64 points) of the SOURCE kd-tree, i.e. 64 queries close
// together in the search space (the pose acts on the 12-D/3-D vectors as an isometry, so
// a leaf stays compact as the source moves).  The wave walks the TARGET kd-tree depth
// first; a node is entered when some lane's f32 box bound is below that lane's pruning
// threshold, and a leaf's <= 64 targets are staged through LDS and swept with broadcast
// ds_read_b128 while each lane keeps (d1, i1, d2).  The previous iteration's match seeds
// the threshold.  The f32 arg-min is then certified (k_loop.hip recheck handles the rest):
//   thr = d1 + 3 err(d1)  => every unvisited target is > 2 err farther than the winner,
//   and among the visited ones the gap d2 - d1 must exceed 2 err(d2).
#include <hip/hip_runtime.h>

#include "loopdev.hpp"
#include "wave.hpp"
#include "tree.hpp"

namespace se3icp {

namespace {

using namespace loopdev;

constexpr int kWaves = 4;
// Leaves wanted by at most this many lanes take the compacted path (8 lanes per query)
#ifndef SE3ICP_NN_COMPACT3
#define SE3ICP_NN_COMPACT3 40  // R3 phase (0: broadcast sweeps only)
#endif
#ifndef SE3ICP_NN_COMPACT
#define SE3ICP_NN_COMPACT 40
#endif

// packed f32 pairs: v_pk_add_f32 / v_pk_fma_f32 issue two lanes' worth of f32 math per
// instruction (the f32 vector peak of gfx950 assumes them)
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int D>
__device__ __forceinline__ float box_lb(const float* lo, const float* hi, const float* q) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float e = fmaxf(fmaxf(lo[d] - q[d], q[d] - hi[d]), 0.f);
        s = fmaf(e, e, s);
    }
    return s;
}

// 12-D: dimensions in pairs on the packed f32 path (v_pk_add_f32 with the box corners
// read as scalar pairs), max(lo - q, q - hi, 0) per dimension (v_max3_f32), v_pk_fma_f32
// chains: 5 instead of 7 VALU per two dimensions
__device__ __forceinline__ float box_lb12(const float* lo, const float* hi, const f32x2* q2) {
    f32x2 s2;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const f32x2 a = f32x2{lo[2 * r], lo[2 * r + 1]} - q2[r];
        const f32x2 b = q2[r] - f32x2{hi[2 * r], hi[2 * r + 1]};
        const f32x2 e = f32x2{fmaxf(fmaxf(a.x, b.x), 0.f), fmaxf(fmaxf(a.y, b.y), 0.f)};
        s2 = (r == 0) ? e * e : __builtin_elementwise_fma(e, e, s2);
    }
    return s2.x + s2.y;
}

// f32 squared 12-D distance of a query (dimension pairs) to a staged target: two
// interleaved FMA chains (even / odd dimensions) and one add, within the D-term chain
// bound f32_err assumes
__device__ __forceinline__ float dist12(const f32x2* q2, const float4* t) {
    const float4 A = t[0], B = t[1], C = t[2];
    f32x2 e, s2;
    e = q2[0] - f32x2{A.x, A.y}; s2 = e * e;
    e = q2[1] - f32x2{A.z, A.w}; s2 = __builtin_elementwise_fma(e, e, s2);
    e = q2[2] - f32x2{B.x, B.y}; s2 = __builtin_elementwise_fma(e, e, s2);
    e = q2[3] - f32x2{B.z, B.w}; s2 = __builtin_elementwise_fma(e, e, s2);
    e = q2[4] - f32x2{C.x, C.y}; s2 = __builtin_elementwise_fma(e, e, s2);
    e = q2[5] - f32x2{C.z, C.w}; s2 = __builtin_elementwise_fma(e, e, s2);
    return s2.x + s2.y;
}

// One leaf against its w wanting queries (list wl): LPQ lanes per query, targets
// sub, sub+LPQ, sub+2LPQ, sub+3LPQ per lane (LPQ * 4 >= cnt), the group's top-2 into
// r1/r2/rb[query].  The lane's 4 targets are loop-invariant over the queries: the
// compiler keeps them in registers (4 waves/SIMD; measured faster than re-reading at 5).
template <int D, int LPQ>
__device__ __forceinline__ void compact_sweep(const float4* tile, const float4* sq, const int* wl, float* r1, float* r2,
                                              int* rb, int w, int cnt, int ta, int lane) {
    constexpr int NV = (D + 3) / 4;
    constexpr int QPI = 64 / LPQ;  // queries per pass
    const int sub = lane & (LPQ - 1);
    for (int it = 0; it < w; it += QPI) {
        const int slot = it + lane / LPQ;
        const int qi = wl[slot < w ? slot : it];
        f32x2 qq[6];
        float4 Q3;
        if constexpr (D == 12) {
            const float4 QA = sq[qi * 3], QB = sq[qi * 3 + 1], QC = sq[qi * 3 + 2];
            qq[0] = f32x2{QA.x, QA.y}; qq[1] = f32x2{QA.z, QA.w}; qq[2] = f32x2{QB.x, QB.y};
            qq[3] = f32x2{QB.z, QB.w}; qq[4] = f32x2{QC.x, QC.y}; qq[5] = f32x2{QC.z, QC.w};
        } else {
            Q3 = sq[qi];
        }
        float a1 = INFINITY, a2 = INFINITY;
        int b1 = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = sub + LPQ * u;
            float acc;
            if constexpr (D == 12) {
                acc = dist12(qq, tile + NV * (j < cnt ? j : 0));
            } else {  // the broadcast sweep's arithmetic (f32_err bound)
                const float4 A = tile[j < cnt ? j : 0];
                float e;
                e = Q3.x - A.x; acc = e * e;
                e = Q3.y - A.y; acc = fmaf(e, e, acc);
                e = Q3.z - A.z; acc = fmaf(e, e, acc);
            }
            acc = j < cnt ? acc : INFINITY;
            const bool lt = acc < a1;
            a2 = __builtin_amdgcn_fmed3f(a1, a2, acc);
            a1 = lt ? acc : a1;
            b1 = lt ? j : b1;
        }
#pragma unroll
        for (int m = 1; m < LPQ; m <<= 1) {
            const float p1 = xor_lane(a1, m), p2 = xor_lane(a2, m);
            const int pb = xor_lane(b1, m);
            const bool lt = (bool)((int)(p1 < a1) | ((int)(p1 == a1) & (int)(pb < b1)));
            a2 = fminf(fmaxf(a1, p1), fminf(a2, p2));
            b1 = lt ? pb : b1;
            a1 = fminf(a1, p1);
        }
        if ((int)(sub == 0) & (int)(slot < w)) {
            r1[qi] = a1;
            r2[qi] = a2;
            rb[qi] = ta + b1;
        }
    }
}

template <int D>
__global__ __launch_bounds__(256) void k_nn_group(View v) {
    constexpr int NV = (D + 3) / 4;
    __shared__ float4 s_tile[kWaves][kLeafMax * NV];
    // compacted leaf sweeps (12-D): the wave's query vectors, the list of lanes that want
    // the current leaf, and the per-query top-2 of the leaf
    __shared__ float4 s_q[kWaves][64 * NV];
    __shared__ int s_wl[kWaves][64];
    __shared__ float s_r1[kWaves][64], s_r2[kWaves][64];
    __shared__ int s_rb[kWaves][64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // wave-uniform work item: the pair record, node boxes and leaf ranges become scalar loads
    const int gi = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + wid);
    if (gi >= v.ngwork) return;
    const GroupWork w = v.gwork[gi];
    const PairDev* P = v.pairs + w.pair;
    const int phase = P->phase;
    if (phase != (D == 12 ? PHASE_SE3 : PHASE_R3)) return;
    const CloudDev cs = v.clouds[P->src], ct = v.clouds[P->tgt];
    const TreeRef TR = (D == 12) ? v.t12 : v.t3;
    const int a = tree_first(cs.n, TR.GL, w.leaf), b = tree_first(cs.n, TR.GL, w.leaf + 1);
    if (b <= a) return;
    const bool valid = lane < b - a;
    const int g = cs.off + (valid ? TR.perm[cs.off + a + lane] : TR.perm[cs.off + a]);

    // query: f64 pose applied to the source element, rounded to f32
    float q[D];
    float na;
    {  // (the f64 query is recomputed at the end rather than held through the traversal)
        double Tm[12], Q[D];
        load_T(P, Tm);
        query_f64<D>(v, Tm, g, Q);
        double n2 = 0;
#pragma unroll
        for (int r = 0; r < D; ++r) {
            const double c = (D == 3) ? Q[r] - P->f32_center[r] : Q[r];
            q[r] = (float)c;
            n2 += c * c;
        }
        na = (float)sqrt(n2) * 1.000001f;
    }
    const float nb = (D == 12) ? P->tgt_norm12 : P->tgt_norm3;
    f32x2 q2[(D + 1) / 2];
#pragma unroll
    for (int r = 0; r < D / 2; ++r) q2[r] = f32x2{q[2 * r], q[2 * r + 1]};
    const float* tv = TR.tvec + ct.off;
    const size_t ld = v.ld;
    if constexpr (D == 12) {
        s_q[wid][lane * 3 + 0] = make_float4(q[0], q[1], q[2], q[3]);
        s_q[wid][lane * 3 + 1] = make_float4(q[4], q[5], q[6], q[7]);
        s_q[wid][lane * 3 + 2] = make_float4(q[8], q[9], q[10], q[11]);
    } else {
        s_q[wid][lane] = make_float4(q[0], q[1], q[2], 0.f);
    }

    float d1 = INFINITY, d2 = INFINITY;
    int i1 = -1;  // target tree position of the best candidate
    float thr = valid ? INFINITY : -1.f;
    if (valid) {  // seed the pruning threshold with the previous match
        const int prev = v.corr_idx[g];
        if (prev >= 0 && prev < ct.n) {
            const int tp = TR.pos[ct.off + prev];
            float s = 0.f;
#pragma unroll
            for (int r = 0; r < D; ++r) {
                const float e = q[r] - tv[(size_t)r * ld + tp];
                s = fmaf(e, e, s);
            }
            thr = s + 3.f * f32_err(s, na, nb, D);
        }
    }

    const float* box_lo = TR.lo + (size_t)P->tgt * TR.nnodes * D;
    const float* box_hi = TR.hi + (size_t)P->tgt * TR.nnodes * D;
    const int first_leaf = (1 << TR.L) - 1;
    float4* tile = s_tile[wid];
    int stk = 0;  // DFS stack in a VGPR: lane i holds entry i (depth <= 2L+1 < 64)
    int sp = 1;
    unsigned n_eval = 0, n_box = 0;  // wave-uniform work counters (roofline accounting)
#ifdef SE3ICP_PROF
    unsigned n_want = 0, n_leafv = 0, n_valid = __popcll(__ballot(valid));
#endif
    while (sp > 0) {
        const int h = __builtin_amdgcn_readlane(stk, sp - 1);
        --sp;
        if (h >= first_leaf) {
            const int li = h - first_leaf;
            const int ta = tree_first(ct.n, TR.L, li), tb = tree_first(ct.n, TR.L, li + 1);
            const int cnt = tb - ta;
            if (cnt <= 0) continue;
            // lanes whose own bound admits this leaf (box re-tested: the bounds shrank since the push)
            unsigned long long W = ~0ull;
            int w = 64;
            if (D == 12 || SE3ICP_NN_COMPACT3) {
                float lbh;
                if constexpr (D == 12) lbh = box_lb12(box_lo + (size_t)h * D, box_hi + (size_t)h * D, q2);
                else lbh = box_lb<D>(box_lo + (size_t)h * D, box_hi + (size_t)h * D, q);
                W = __ballot(lbh * (1.f - 2e-6f) < thr);
                if (W == 0ull) continue;
                w = __popcll(W);
            }
#ifdef SE3ICP_PROF
            n_want += __popcll(W & __ballot(valid));
            ++n_leafv;
#endif
            __builtin_amdgcn_wave_barrier();
            if (lane < cnt) {
                float e[NV * 4];
#pragma unroll
                for (int r = 0; r < NV * 4; ++r) e[r] = (r < D) ? tv[(size_t)r * ld + ta + lane] : 0.f;
#pragma unroll
                for (int k = 0; k < NV; ++k) tile[lane * NV + k] = make_float4(e[4 * k], e[4 * k + 1], e[4 * k + 2], e[4 * k + 3]);
            }
            __builtin_amdgcn_wave_barrier();
            if (w > (D == 12 ? SE3ICP_NN_COMPACT : SE3ICP_NN_COMPACT3)) {
                // every lane sweeps every target (broadcast LDS reads)
                for (int j = 0; j < cnt; ++j) {
                    float acc;
                    if constexpr (D == 12) {
                        acc = dist12(q2, tile + j * 3);
                    } else {
                        const float4 A = tile[j];
                        float e;
                        e = q[0] - A.x; acc = e * e;
                        e = q[1] - A.y; acc = fmaf(e, e, acc);
                        e = q[2] - A.z; acc = fmaf(e, e, acc);
                    }
                    const bool lt = acc < d1;
                    d2 = __builtin_amdgcn_fmed3f(d1, d2, acc);
                    d1 = lt ? acc : d1;
                    i1 = lt ? (ta + j) : i1;  // target tree position
                }
                n_eval += cnt;
            } else {
                // compacted: LPQ lanes per wanting query (8 for leaves of <= 32 targets, 16
                // up to 64), 4 targets per lane, then a top-2 merge over the LPQ lanes and
                // into the query's own lane
                if ((W >> lane) & 1ull)
                    s_wl[wid][__builtin_amdgcn_mbcnt_hi((unsigned)(W >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)W, 0u))] = lane;
                __builtin_amdgcn_wave_barrier();
                if (cnt <= 32) compact_sweep<D, 8>(tile, s_q[wid], s_wl[wid], s_r1[wid], s_r2[wid], s_rb[wid], w, cnt, ta, lane);
                else compact_sweep<D, 16>(tile, s_q[wid], s_wl[wid], s_r1[wid], s_r2[wid], s_rb[wid], w, cnt, ta, lane);
                __builtin_amdgcn_wave_barrier();
                if ((W >> lane) & 1ull) {
                    const float r1 = s_r1[wid][lane], r2 = s_r2[wid][lane];
                    const int rb = s_rb[wid][lane];
                    d2 = fminf(fmaxf(d1, r1), fminf(d2, r2));
                    i1 = r1 < d1 ? rb : i1;
                    d1 = fminf(d1, r1);
                }
                __builtin_amdgcn_wave_barrier();
                n_eval += 4 * ((w + (cnt <= 32 ? 7 : 3)) >> (cnt <= 32 ? 3 : 2));  // 64-lane evaluation slots issued
            }
            if ((int)valid & (int)(d1 < INFINITY)) thr = fminf(thr, d1 + 3.f * f32_err(d1, na, nb, D));
            continue;
        }
        n_box += 2;
        const int hl = 2 * h + 1, hr = 2 * h + 2;
        float ll, lr;
        if constexpr (D == 12) {
            ll = box_lb12(box_lo + (size_t)hl * D, box_hi + (size_t)hl * D, q2);
            lr = box_lb12(box_lo + (size_t)hr * D, box_hi + (size_t)hr * D, q2);
        } else {
            ll = box_lb<D>(box_lo + (size_t)hl * D, box_hi + (size_t)hl * D, q);
            lr = box_lb<D>(box_lo + (size_t)hr * D, box_hi + (size_t)hr * D, q);
        }
        // the f32 bound is within (D+2) ulps of the exact distance to the (inflated) box
        const bool vl = __ballot(ll * (1.f - 2e-6f) < thr) != 0ull;
        const bool vr = __ballot(lr * (1.f - 2e-6f) < thr) != 0ull;
        const bool left_first = __builtin_amdgcn_readfirstlane(ll <= lr ? 1 : 0) != 0;
        const int nearh = left_first ? hl : hr, farh = left_first ? hr : hl;
        const bool vnear = left_first ? vl : vr, vfar = left_first ? vr : vl;
        if (vfar) { stk = (lane == sp) ? farh : stk; ++sp; }
        if (vnear) { stk = (lane == sp) ? nearh : stk; ++sp; }
    }

    if (lane == 0) {  // 64 lanes per evaluation; 64 counter slots against contention
        unsigned long long* st = v.stats + kStatCols * (gi & 63) + (D == 12 ? 0 : 2);
        atomicAdd(st, 64ull * n_eval);
        atomicAdd(st + 1, 64ull * n_box);
#ifdef SE3ICP_PROF
        if (D == 12) {
            atomicAdd(v.stats + kStatCols * (gi & 63) + 8, (unsigned long long)n_want);
            atomicAdd(v.stats + kStatCols * (gi & 63) + 9, (unsigned long long)n_leafv);
            atomicAdd(v.stats + kStatCols * (gi & 63) + 10, (unsigned long long)n_leafv * n_valid);
        }
#endif
    }
    if (!valid) return;
    // certification (see the header) and the stored distance
    const bool flag = (bool)((int)(i1 < 0) | (int)!(d2 - d1 > 2.f * f32_err(d2, na, nb, D)));
    if ((int)flag & (int)(ct.n > 1)) {
        const int at = atomicAdd(v.flag_count, 1);
        v.flag_list[at] = g;
        atomicAdd(&v.pair_rechecked[w.pair], 1);
    }
    // tree position -> target index; a NaN query keeps the reference's zero-initialised index
    i1 = (i1 < 0) ? 0 : TR.perm[ct.off + i1];
    v.corr_idx[g] = i1;
    double Tm[12], Q[D];
    load_T(P, Tm);
    query_f64<D>(v, Tm, g, Q);
    if constexpr (D == 12) {
        v.corr_dist[g] = stored_dist(v, PHASE_SE3, ct, Q, i1);
    } else {
        double Q12[12];
        Q12[0] = Q[0]; Q12[1] = Q[1]; Q12[2] = Q[2];
        v.corr_dist[g] = stored_dist(v, PHASE_R3, ct, Q12, i1);
    }
}

}  // namespace

void launch_nn_se3(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_nn_group<12>, dim3((v.ngwork + kWaves - 1) / kWaves), dim3(64 * kWaves), 0, s, v);
}
void launch_nn_r3(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_nn_group<3>, dim3((v.ngwork + kWaves - 1) / kWaves), dim3(64 * kWaves), 0, s, v);
}

}  // namespace se3icp
