// MI355X (gfx950) kernel for the restricted decision diagram of SGUFP_Solver:
// Inavap::RestrictedDDNew (/root/reference/DD.cpp:3090-3505) under the restricted cut
// phases of NodeExplorer::processX3 (NodeExplorer.cpp:605-656).
//
// One 64-lane wave per open node:
//   1. compile (DD.cpp:3090-3159, 3222-3260, 3161-3220): the tree expands exactly -- each
//      node's states in reverse stored order, child states = parent minus the decision (-1
//      keeps all) -- until a layer would exceed `width` (<= 128) nodes; that layer keeps its
//      first `width` children and from then on every node has one child whose decision is
//      its largest state.  Layers live as u32 state masks in LDS; each node's (parent, rank)
//      word goes to HBM for the path walks.
//   2. sweeps of the pool's cuts, CB = 4 at a time (feasibility list then optimality list,
//      newest first): the tree part layer by layer through LDS, the single-child part
//      ("chains") in registers with the decisions replayed from the state masks; only leaf
//      values are needed, since only last-layer nodes are ever removed (DD.cpp:3340-3423).
//   3. the per-cut replay in pool order: feasibility -- leaves with state2 < -0.5 lose their
//      terminal arc, no leaf left -> infeasible; optimality -- terminal weights take the
//      running minimum and the bound is their maximum (DD.cpp:3425-3505); a bound <=
//      optimalLB ends the node (NodeExplorer.cpp:635-647).
//   4. the max path (getMaxPath, DD.cpp:3290-3305) and, for a non-exact tree, the exact
//      cutset (getExactCutSet, DD.cpp:3279-3288).
// Bit-exactness: the same IEEE adds in the same order as the reference's sequential folds,
// -ffp-contract=off; std::min / std::max ties as the reference (zero maxima recomputed with
// the (value, priority) pick).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "dd_device.hpp"
#include "rdd_device.hpp"
#include "wave.hpp"

namespace sgufp {

namespace {

#define DMIN (-__DBL_MAX__)
#define DMAX (__DBL_MAX__)

constexpr int RCB = 4;                       // cuts per sweep
constexpr int RG = kWave / RCB;              // node groups per wave
constexpr int RU = kRddMax / RG;             // nodes per lane (8)
constexpr int kChainBlock = 4;               // chain layers whose coefficients load together

struct RLds {
    LDS int16_t *rslot;    // [Lcap] coefficient slot of each root-solution decision
    LDS uint32_t *cm;      // [2][kRddMax] state masks of the current / next layer
    LDS double *vb;        // [2][kRddMax][RCB] values of the tree part
    LDS uint8_t *lw;       // [Tcap] layer widths
    LDS double *ct;        // [RCB][us] coefficients of the layer being swept (tree part)
    LDS int32_t *ids;      // [RCB] pool rows of the batch
};

__host__ __device__ inline size_t ra16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline size_t rlds_layout(int Tcap, int Lcap, int us, size_t *off) {
    size_t o = 0;
    off[0] = o; o = ra16(o + (size_t)Lcap * 2);
    off[1] = o; o = ra16(o + (size_t)2 * kRddMax * 4);
    off[2] = o; o = ra16(o + (size_t)2 * kRddMax * RCB * 8);
    off[3] = o; o = ra16(o + (size_t)Tcap);
    off[4] = o; o = ra16(o + (size_t)RCB * us * 8);
    off[5] = o; o = ra16(o + (size_t)RCB * 4);
    return o;
}

__device__ __forceinline__ double rsmin(double a, double b) { return (b < a) ? b : a; }  // std::min
__device__ __forceinline__ double rsmax(double a, double b) { return (a < b) ? b : a; }  // std::max
// largest state of a mask (states are stored ascending, -1 = rank 0 first); 0 for an empty mask
__device__ __forceinline__ uint32_t hibit(uint32_t m) { return m ? 31u - (uint32_t)__clz(m) : 0u; }

__device__ __forceinline__ int16_t rvalue(const NetDev &net, int layer, int r) {
    return net.set_val[net.set_off[net.layer_universe[layer]] + r];
}

// Coefficient of state rank r at tree layer k for pool row id.  The structural layer (the
// decision's state set) is g + k - 1; the coefficient layer (the key's (q, i)) is the
// reference's running index len + k - 1 (DD.cpp:3346-3374); they differ only for records
// whose solution vector is shorter than their global layer.
struct Coef {
    const NetDev *net;
    const Pool *pool;
    int g, len, aligned;
    size_t ltab;
    __device__ __forceinline__ double operator()(int id, int k, uint32_t r) const {
        if (r == 0) return 0.0;
        if (aligned) return pool->coefT[(size_t)id * ltab + (size_t)(g + k - 1) * pool->ustride + r];
        const int dec = rvalue(*net, g + k - 1, (int)r);
        if (dec < 0) return 0.0;
        const int lc = len + k - 1, j = net->arc_head[dec];
        int s = net->n_slots;
        for (int q = net->slot_off[lc]; q < net->slot_off[lc + 1]; q++)
            if (net->slot_head[q] == j) { s = q; break; }
        return pool->rows[(size_t)id * pool->stride + s];
    }
};

__device__ __forceinline__ double rfold(const GBL double *row, double v, const LDS int16_t *rslot, int len) {
    constexpr int B = 16;
    for (int t0 = 0; t0 < len; t0 += B) {
        double x[B];
        bool ok[B];
#pragma unroll
        for (int j = 0; j < B; j++) {
            const int t = t0 + j;
            const int sl = t < len ? (int)rslot[t] : -1;
            ok[j] = sl >= 0;
            x[j] = row[ok[j] ? sl : 0];
        }
        sched_fence();
#pragma unroll
        for (int j = 0; j < B; j++)
            if (ok[j]) v = v + x[j];
    }
    return v;
}

}  // namespace

__global__ void __launch_bounds__(kWave, 2) k_restrict(NetDev net, BatchIn in, Pool pool, RddIO io, double optimal_lb) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS uint8_t *smem = (LDS uint8_t *)smem_raw;
    const int slot = blockIdx.x;
    if (slot >= in.n) return;
    size_t off[6];
    rlds_layout(io.Tcap, io.Lcap, pool.ustride, off);
    RLds W;
    W.rslot = (LDS int16_t *)(smem + off[0]);
    W.cm = (LDS uint32_t *)(smem + off[1]);
    W.vb = (LDS double *)(smem + off[2]);
    W.lw = (LDS uint8_t *)(smem + off[3]);
    W.ct = (LDS double *)(smem + off[4]);
    W.ids = (LDS int32_t *)(smem + off[5]);

    const int g = uni((int)in.gl[slot]), len = uni((int)in.sol_len[slot]);
    const GBL int16_t *rsol = in.sol + in.sol_off[slot];
    GBL uint16_t *topo = io.topo + (size_t)slot * io.Tcap * kRddMax;
    const int Wd = io.width;
    int status = kSuccess;
    int exact = 1, E = 0, T = 1;
    double lower = in.lb[slot];
    if (!in.valid[slot] || len > g || g > net.L || len > io.Lcap || net.L + 1 > io.Tcap) {
        status = kErrRecord;
        goto done;
    }
    // coefficient slots of the root solution (layer t, decision sol[t])
    for (int t = lane(); t < len; t += kWave) {
        const int dec = rsol[t];
        int s = -1;
        if (dec != -1) {
            s = net.n_slots;
            if (dec >= 0 && dec < net.m) {
                const int j = net.arc_head[dec];
                for (int q = net.slot_off[t]; q < net.slot_off[t + 1]; q++)
                    if (net.slot_head[q] == j) { s = q; break; }
            }
        }
        W.rslot[t] = (int16_t)s;
    }
    // ---- 1. compile
    {
        if (lane() == 0) { W.cm[0] = in.mask[slot]; W.lw[0] = 1; }
        wave_lds_sync();
        uint32_t w = 1;
        int cur = 0;
        for (int a = g; a < net.L; a++) {
            const int idx = a - g;
            LDS uint32_t *cmk = W.cm + cur * kRddMax, *nmk = W.cm + (cur ^ 1) * kRddMax;
            GBL uint16_t *tk = topo + (size_t)(idx + 1) * kRddMax;
            const int upd = net.layer_update[a];
            if (upd >= 0) {   // stateUpdateMap: every current-layer node takes the full set
                const int sl = net.set_len[upd];
                const uint32_t full = (sl >= 32) ? 0xFFFFFFFFu : ((1u << sl) - 1u);
                for (uint32_t i = lane(); i < w; i += kWave) cmk[i] = full;
                wave_lds_sync();
            }
            uint32_t wn;
            if (exact) {
                uint32_t carry = 0;
                for (uint32_t base = 0; base < w; base += kWave) {
                    const uint32_t i = base + lane();
                    const uint32_t m = i < w ? cmk[i] : 0u;
                    const uint32_t c = __popc(m);
                    const uint32_t incl = wave_scan_incl(c);
                    uint32_t j = carry + incl - c;
                    // children in reverse stored order: largest state first
                    for (uint32_t mm = m; mm && j < (uint32_t)Wd; j++) {
                        const uint32_t r = hibit(mm);
                        mm &= ~(1u << r);
                        nmk[j] = (r == 0) ? m : (m & ~(1u << r));
                        tk[j] = (uint16_t)(i | (r << 7));
                    }
                    carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
                }
                if (carry > (uint32_t)Wd) {
                    // RestrictedDDNew::buildNextLayer stops at `width` children: not exact
                    // from here; the current layer is the exact cutset layer E
                    exact = 0;
                    wn = (uint32_t)Wd;
                    for (uint32_t i = lane(); i < w; i += kWave) io.csm[(size_t)slot * kRddMax + i] = cmk[i];
                } else {
                    wn = carry;
                    E++;
                }
            } else {
                for (uint32_t i = lane(); i < w; i += kWave) {
                    const uint32_t m = cmk[i];
                    const uint32_t r = hibit(m);
                    nmk[i] = (r == 0) ? m : (m & ~(1u << r));
                    tk[i] = (uint16_t)(i | (r << 7));
                }
                wn = w;
            }
            wave_lds_sync();
            // the masks the chain replay starts from: layer E + 1, the first one built after
            // the exact part ended
            if (!exact && idx + 1 == E + 1)
                for (uint32_t i = lane(); i < wn; i += kWave) io.cmask[(size_t)slot * kRddMax + i] = nmk[i];
            if (lane() == 0) W.lw[idx + 1] = (uint8_t)(wn == 256 ? 255 : wn);
            w = wn;
            cur ^= 1;
            T++;
        }
        wave_mem_sync();
    }
    {
        // ---- 2./3. sweeps and the per-cut replay
        const int TR = exact ? T - 1 : min(E + 1, T - 1);     // last layer of the tree part
        const int c = lane() % RCB, grp = lane() / RCB;
        const Coef coef{&net, &pool, g, len, len == g ? 1 : 0, (size_t)net.L * pool.ustride};
        const uint32_t wl = uni((uint32_t)W.lw[T - 1]) == 255 ? 256u : uni((uint32_t)W.lw[T - 1]);
        // leaves in lane order: leaf lane and lane + 64; alive bits per half
        uint64_t al0 = wl >= 64 ? ~0ull : ((1ull << wl) - 1ull);
        uint64_t al1 = wl > 64 ? (wl >= 128 ? ~0ull : ((1ull << (wl - 64)) - 1ull)) : 0ull;
        double tw0 = DMAX, tw1 = DMAX;
        const int total = pool.nf + pool.no;
        LDS double *leafv = W.vb + (size_t)(T & 1) * kRddMax * RCB;    // after the sweep: [leaf][c]
        for (int s = 0; s < total && status == kSuccess;) {
            const bool feas = s < pool.nf;
            const int nb = min(RCB, (feas ? pool.nf : total) - s);
            if (lane() < RCB) W.ids[lane()] = (lane() < nb) ? (s + lane() < pool.nf ? pool.f_order[s + lane()]
                                                                                  : pool.o_order[s + lane() - pool.nf])
                                                            : 0;
            wave_lds_sync();
            const int id = W.ids[c];
            const double rv = rfold(pool.rows + (size_t)id * pool.stride, pool.rhs[id], W.rslot, len);
            // tree part through LDS
            if (lane() < RCB) W.vb[c] = rv;
            wave_lds_sync();
            for (int k = 1; k <= TR; k++) {
                const uint32_t wk = uni((uint32_t)W.lw[k]) == 255 ? 256u : uni((uint32_t)W.lw[k]);
                // RCB * ustride entries: up to 4 x 32 (network.cpp admits 32 states per set),
                // more than the wave's lanes
                for (int e = lane(); e < RCB * pool.ustride; e += kWave) {
                    const int cc = e / pool.ustride, r = e - cc * pool.ustride;
                    W.ct[cc * pool.ustride + r] = coef(W.ids[cc], k, (uint32_t)r);
                }
                wave_lds_sync();
                const LDS double *pv = W.vb + (size_t)((k - 1) & 1) * kRddMax * RCB;
                LDS double *nv = W.vb + (size_t)(k & 1) * kRddMax * RCB;
                const GBL uint16_t *tk = topo + (size_t)k * kRddMax;
                uint32_t wd[RU];
#pragma unroll
                for (int u = 0; u < RU; u++) {
                    const uint32_t i = (uint32_t)(grp + u * RG);
                    wd[u] = i < wk ? (uint32_t)tk[i] : 0u;
                }
                sched_fence();
                double px[RU], cf[RU];
#pragma unroll
                for (int u = 0; u < RU; u++) {
                    px[u] = pv[(wd[u] & 127u) * RCB + c];
                    cf[u] = W.ct[c * pool.ustride + (wd[u] >> 7)];
                }
                sched_fence();
#pragma unroll
                for (int u = 0; u < RU; u++) {
                    const uint32_t i = (uint32_t)(grp + u * RG);
                    if (i < wk) nv[i * RCB + c] = (wd[u] >> 7) != 0 ? px[u] + cf[u] : px[u];
                }
                wave_lds_sync();
            }
            if (TR < T - 1) {
                // chains: node i keeps index i; the decision is the largest state of its mask
                double x[RU];
                uint32_t mk[RU];
                const LDS double *pv = W.vb + (size_t)(TR & 1) * kRddMax * RCB;
#pragma unroll
                for (int u = 0; u < RU; u++) {
                    const uint32_t i = (uint32_t)(grp + u * RG);
                    x[u] = i < wl ? pv[i * RCB + c] : 0.0;
                    mk[u] = i < wl ? io.cmask[(size_t)slot * kRddMax + i] : 1u;
                }
                for (int k0 = TR + 1; k0 < T; k0 += kChainBlock) {
                    uint32_t rk[kChainBlock][RU];
                    double cf[kChainBlock][RU];
#pragma unroll
                    for (int b = 0; b < kChainBlock; b++) {
                        const int k = k0 + b;
                        const bool okk = k < T;
                        const int upd = okk ? net.layer_update[g + k - 1] : -1;
                        uint32_t full = 0;
                        if (upd >= 0) {
                            const int sl = net.set_len[upd];
                            full = (sl >= 32) ? 0xFFFFFFFFu : ((1u << sl) - 1u);
                        }
#pragma unroll
                        for (int u = 0; u < RU; u++) {
                            if (upd >= 0) mk[u] = full;
                            const uint32_t r = okk ? hibit(mk[u]) : 0u;
                            rk[b][u] = r;
                            mk[u] = (r == 0) ? mk[u] : (mk[u] & ~(1u << r));
                            cf[b][u] = okk ? coef(id, k, r) : 0.0;
                        }
                    }
                    sched_fence();
#pragma unroll
                    for (int b = 0; b < kChainBlock; b++)
#pragma unroll
                        for (int u = 0; u < RU; u++) x[u] = rk[b][u] != 0 ? x[u] + cf[b][u] : x[u];
                }
#pragma unroll
                for (int u = 0; u < RU; u++) {
                    const uint32_t i = (uint32_t)(grp + u * RG);
                    if (i < wl) leafv[i * RCB + c] = x[u];
                }
            } else if (T - 1 == 0) {
                if (lane() < RCB) leafv[c] = rv;
            } else if (((T - 1) & 1) != (T & 1)) {
                // the last tree layer is in buffer (T-1)&1; leafv is the other one
                const LDS double *pv = W.vb + (size_t)((T - 1) & 1) * kRddMax * RCB;
#pragma unroll
                for (int u = 0; u < RU; u++) {
                    const uint32_t i = (uint32_t)(grp + u * RG);
                    if (i < wl) leafv[i * RCB + c] = pv[i * RCB + c];
                }
            }
            wave_lds_sync();
            // replay in pool order; leaf lane / lane + 64
            for (int cc = 0; cc < nb && status == kSuccess; cc++) {
                const double v0 = leafv[(size_t)lane() * RCB + cc];
                const double v1 = leafv[(size_t)(lane() + 64) * RCB + cc];
                if (feas) {
                    if (!(al0 | al1)) { status = kPrunedFeasibility; break; }
                    al0 &= ~__ballot(v0 < -0.5);
                    al1 &= ~__ballot(v1 < -0.5);
                    if (!(al0 | al1)) { status = kPrunedFeasibility; break; }
                } else {
                    const bool a0 = (al0 >> lane()) & 1ull, a1 = (al1 >> lane()) & 1ull;
                    if (a0) tw0 = rsmin(tw0, v0);
                    if (a1) tw1 = rsmin(tw1, v1);
                    double mx = -INFINITY;
                    if (a0) mx = tw0;
                    if (a1) mx = (tw1 > mx) ? tw1 : mx;
                    mx = lane_reduce<1>(mx, [](double p, double q) { return (q > p) ? q : p; });
                    double term;
                    if (mx == -INFINITY) term = DMIN;
                    else if (mx != 0.0) term = rsmax(DMIN, mx);
                    else {
                        // a zero maximum: the first leaf holding it decides the sign (old wins)
                        const uint64_t b0 = __ballot(a0 && tw0 == 0.0), b1 = __ballot(a1 && tw1 == 0.0);
                        const int first = b0 ? (int)__ffsll((unsigned long long)b0) - 1
                                             : 64 + (int)__ffsll((unsigned long long)b1) - 1;
                        const double z = first < 64 ? lane_get(tw0, first) : lane_get(tw1, first - 64);
                        term = rsmax(DMIN, z);
                    }
                    lower = term;
                    if (lower <= optimal_lb) { status = kPrunedOptimality; break; }
                }
            }
            s += nb;
            wave_lds_sync();
        }
        // ---- 4. max path and cutset
        if (lane() == 0) {
            io.status[slot] = status;
            io.exact[slot] = (uint8_t)exact;
            io.lb[slot] = lower;
        }
        GBL int16_t *path = io.path + (size_t)slot * io.Lcap;
        int plen = 0;
        if (status == kSuccess) {
            // strict > from DOUBLE_MIN over the alive leaves in order: the first maximum
            const bool a0 = (al0 >> lane()) & 1ull, a1 = (al1 >> lane()) & 1ull;
            double mx = DMIN;
            if (a0 && tw0 > mx) mx = tw0;
            if (a1 && tw1 > mx) mx = tw1;
            mx = lane_reduce<1>(mx, [](double p, double q) { return (q > p) ? q : p; });
            int best = -1;
            if (mx > DMIN) {
                const uint64_t b0 = __ballot(a0 && tw0 == mx), b1 = __ballot(a1 && tw1 == mx);
                best = b0 ? (int)__ffsll((unsigned long long)b0) - 1 : 64 + (int)__ffsll((unsigned long long)b1) - 1;
            }
            for (int t = lane(); t < len; t += kWave) path[t] = rsol[t];
            if (best >= 0) {
                // chain part: the node index stays the leaf's
                for (int k = TR + 1 + lane(); k < T; k += kWave) {
                    const uint32_t wd = topo[(size_t)k * kRddMax + best];
                    path[len + k - 1] = rvalue(net, g + k - 1, (int)(wd >> 7));
                }
                // tree part: walk the parents up
                if (lane() == 0) {
                    uint32_t node = (uint32_t)best;
                    for (int k = TR; k >= 1; k--) {
                        const uint32_t wd = topo[(size_t)k * kRddMax + node];
                        path[len + k - 1] = rvalue(net, g + k - 1, (int)(wd >> 7));
                        node = wd & 127u;
                    }
                }
                plen = len + T - 1;
            } else {
                plen = len;
            }
        }
        if (lane() == 0) io.path_len[slot] = (uint16_t)plen;
        // exact cutset (getExactCutSet): nodes of layer E, their decisions from the root
        const uint32_t wE = uni((uint32_t)W.lw[E]) == 255 ? 256u : uni((uint32_t)W.lw[E]);
        if (lane() == 0) {
            io.cs_n[slot] = exact ? 0u : wE;
            io.cs_gl[slot] = (uint16_t)(g + E);
        }
        if (!exact) {
            for (uint32_t j = lane(); j < wE; j += kWave) {
                GBL int16_t *dec = io.csdec + ((size_t)slot * kRddMax + j) * io.Tcap;
                uint32_t node = j;
                for (int k = E; k >= 1; k--) {
                    const uint32_t wd = topo[(size_t)k * kRddMax + node];
                    dec[k - 1] = rvalue(net, g + k - 1, (int)(wd >> 7));
                    node = wd & 127u;
                }
            }
        }
        return;
    }
done:
    if (lane() == 0) {
        io.status[slot] = status;
        io.exact[slot] = (uint8_t)exact;
        io.lb[slot] = DMIN;
        io.path_len[slot] = 0;
        io.cs_n[slot] = 0;
        io.cs_gl[slot] = 0;
    }
}

size_t rdd_lds_bytes(int Tcap, int Lcap, int us) {
    size_t off[6];
    return rlds_layout(Tcap, Lcap, us, off);
}

hipError_t launch_restrict(const NetDev &net, const BatchIn &in, const Pool &pool, const RddIO &io, double optimal_lb,
                           hipStream_t st) {
    if (in.n <= 0) return hipSuccess;
    const size_t lds = rdd_lds_bytes(io.Tcap, io.Lcap, pool.ustride);
    hipLaunchKernelGGL(k_restrict, dim3(in.n), dim3(kWave), lds, st, net, in, pool, io, optimal_lb);
    return hipGetLastError();
}

}  // namespace sgufp
