// MI355X (gfx950) kernels for the per-B&B-node relaxation of SGUFP_Solver.
//
// One open node = one relaxed decision diagram = one 64-lane wavefront (a single-wave
// workgroup).  Per node the kernel
//   1. builds the relaxed DD layer by layer (RelaxedDDNew::buildTree / buildNextLayer,
//      /root/reference/DD.cpp:3528-3694): wave prefix scans give child offsets, state
//      sets are u32 masks over the V-bar node's sorted state universe;
//   2. sweeps every pool cut over it (applyFeasibilityCut DD.cpp:3842-3930,
//      applyOptimalityCut DD.cpp:3932-4023): a layered (max,+) longest path whose
//      previous-layer state2 lives in LDS; coefficients come from dense cut rows
//      (one slot per (layer, head) key, Cut.h:275-282/342-344) gathered once per layer
//      by 32 lanes and broadcast by rank;
//   3. applies the reference's edits exactly: last-layer removal with the bottom-up
//      deletion cascade (DD.cpp:4040-4119), width-1 arc pruning (DD.cpp:3895-3928,
//      3987-4021), running-min terminal weights;
//   4. finishes like NodeExplorer::process (NodeExplorer.cpp:915-986): the cutset
//      layer and child count (getCutset, DD.cpp:4179-4218) or, for an exact DD, the
//      argmax path (getSolution, DD.cpp:3825-3840) for the scenario subproblem.
// A second kernel writes the cutset children as frontier records.
//
// Bit-exactness: only IEEE adds, compares and std::max/std::min-style selects are used,
// in the reference's order (ties resolved exactly like the sequential folds); the file is
// compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "dd_device.hpp"
#include "wave.hpp"

namespace sgufp {

// Address spaces spelled out so that the compiler emits ds_* for LDS and global_* for
// HBM: a generic (flat) access waits on both counters and serialises LDS behind HBM.
#define DMIN (-__DBL_MAX__)
#define DMAX (__DBL_MAX__)

constexpr uint32_t kCollapseWidth = 120;  // RELAXED_MAX_WIDTH (DD.h:732)


// (value, priority) arg-max.  A sequential std::max fold keeps either the newer or the
// older of two equal values; equal doubles differ only in the sign of zero, and the
// priority reproduces which one the fold would keep.
struct VP {
    double v;
    int p;  // INT_MIN = empty
};
__device__ __forceinline__ VP vp_pick(VP a, VP b) {
    // branch-free: selects only (this sits in the innermost sweep loops)
    const bool take_b = (a.p == INT_MIN) | ((b.p != INT_MIN) & ((b.v > a.v) | (!(a.v > b.v) & (b.p > a.p))));
    VP r;
    r.v = take_b ? b.v : a.v;
    r.p = take_b ? b.p : a.p;
    return r;
}
template <int S0 = 1>
__device__ __forceinline__ VP wave_vp(VP x) {
    if constexpr (S0 < kWave) {
        VP y;
        y.v = lane_x<S0>(x.v);
        y.p = lane_x<S0>(x.p);
        return wave_vp<S0 * 2>(vp_pick(x, y));
    } else {
        return x;
    }
}
__device__ __forceinline__ double wave_fmin(double x) {
    return lane_reduce<1>(x, [](double a, double b) { return fmin(a, b); });
}
// fold "acc = max(x_k, acc)" (new element wins ties) -> priority k;
// fold "acc = max(acc, x_k)" (old element wins ties) -> priority -k-2.
__device__ __forceinline__ int prio_new(int k) { return k; }
__device__ __forceinline__ int prio_old(int k) { return -k - 2; }

// ------------------------------------------------------------------------------------
// Per-DD view: the layer table lives in LDS for the lifetime of the kernel, the
// node/arc arrays in this slot's HBM scratch.
struct DD {
    // LDS
    LDS uint32_t *noff, *nn, *nalive, *aoff, *acnt;
    LDS int16_t *rslot;   // [Lcap] coefficient slot of each root-solution decision (-1: decision -1)
    LDS double *buf0, *buf1;
    LDS double *coef;     // [us] per-rank coefficients of the layer being swept
    LDS int16_t *walk;    // [Tcap] decisions collected by a path walk
    GBL double *sm1;      // [Tcap] width-1 layers: state2 of the single node (last single sweep)
    GBL double *xm1;      // [Tcap] width-1 layers: min over its in-arcs of parent.state2 + weight
    GBL uint8_t *v1;      // [Tcap] summary valid (layer had one alive node during that sweep)
    int us;               // entries of the per-layer coefficient tables
    // HBM (slot base applied)
    GBL uint32_t *ntopo;
    GBL uint8_t *nflag;
    GBL uint32_t *nmask;
    GBL uint32_t *outcnt;
    GBL double *s2;
    GBL double *tw;
    GBL uint32_t *atopo;
    GBL uint8_t *aflag;
    GBL uint16_t *tmir;   // packed topology of the narrow layers (see build_stream)
    LDS uint16_t *gstart; // [Tcap] first layer of each staging group of the narrow sweep
    // scalars
    int g, len, T, exact, aligned;
    int kg;           // first layer wider than kLdsBatchWidth (or the last layer)
    uint32_t Nn;      // nodes in layers < kg (packed node words)
    uint32_t Amir;    // merged-layer arcs (all in layers < kg)
    int stream;       // packed topology valid
    int ng;           // staging groups of layers 1 .. kg-1
};

constexpr int kLdsBatchWidth = 128;
constexpr int kStageEntries = 128;   // coefficient staging ring: f64 entries per slot (2 per lane)
constexpr int kTopoEntries = 512;    // topology staging ring: u16 entries per slot (8 per lane)
constexpr int kStageLayers = 16;     // at most this many layers per staging group
constexpr int kMaxRun = 5;           // exact layers folded in registers per narrow-sweep step (odd)
constexpr uint32_t kNarrowMax = 127;  // widest narrow layer; value slot 127 holds the NaN sentinel

// Packed topology of the narrow layers (HBM, per DD slot): node word = parent:7 | rank:5 |
// alive | in-arc alive for nodes [0, Nn), merged-arc word = parent:7 | rank:5 | alive for
// arcs at Nn + [0, Amir).  Layers are contiguous in both ranges, so the words of a run of
// layers are two contiguous segments that the narrow sweep stages into LDS ahead of use.
// ntopo / nflag / atopo / aflag stay the master copy; every edit of a narrow node / arc
// flag is applied to both.
// Parent slot / rank field of a packed topology word as single bit-field instructions (the
// compiler's shift-then-mask canonical form costs a third instruction per address).
static_assert(kMirParent == 127 && kMirRankShift == 7, "mir_parent / mir_rank encode the field positions");
__device__ __forceinline__ uint32_t mir_parent(uint32_t w) {
    uint32_t r;
    asm("v_and_b32 %0, 0x7f, %1" : "=v"(r) : "v"(w));
    return r;
}
__device__ __forceinline__ uint32_t mir_rank(uint32_t w) {
    uint32_t r;
    asm("v_bfe_u32 %0, %1, 7, 5" : "=v"(r) : "v"(w));
    return r;
}
__device__ __forceinline__ void mir_node_clear(DD &d, uint32_t node, uint16_t bits) {
    if (d.stream && node < d.Nn) d.tmir[node] &= (uint16_t)~bits;
}
__device__ __forceinline__ void mir_arc_kill(DD &d, uint32_t a, uint32_t rank) {
    if (d.stream) d.tmir[d.Nn + a] = (uint16_t)(kNarrowMax | ((rank & 31u) << kMirRankShift));
}
__device__ __forceinline__ void mir_arc_clear(DD &d, uint32_t a) {
    // dead: no alive bit, parent slot = the NaN sentinel of the narrow sweep
    if (d.stream) d.tmir[d.Nn + a] = (uint16_t)((d.tmir[d.Nn + a] & ~(kMirAlive | kMirParent)) | kNarrowMax);
}

struct LdsCarve {
    size_t bytes;
    size_t o_lay, o_rslot, o_buf, o_coef, o_walk, o_bcoef, o_w1, o_ids, o_sm1, o_xm1, o_v1, o_gs, o_ring, o_tring, o_wm;
};

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// cb = cuts per batched sweep (1 = single-cut kernels only), us = coefficient entries per
// layer.  At 1k arcs (L = 281, us = 5, cb = 4) this is 20 KB: eight waves per CU.
__host__ __device__ inline LdsCarve lds_carve(int Tcap, int Lcap, int cb, int us) {
    LdsCarve c;
    size_t o = 0;
    size_t single = (size_t)2 * kLdsWidth * 8, batch = (size_t)2 * 128 * (cb > 1 ? cb : 0) * 8;
    c.o_lay = o; o = align16(o + (size_t)Tcap * 5 * 4);
    c.o_rslot = o; o = align16(o + (size_t)Lcap * 2);
    c.o_buf = o; o = align16(o + (single > batch ? single : batch));
    c.o_coef = o; o = align16(o + (size_t)us * 8);
    c.o_walk = o; o = align16(o + (size_t)Tcap * 2);
    c.o_bcoef = o; o = align16(o + (cb > 1 ? (size_t)cb * us * 8 : 0));
    c.o_w1 = o; o = align16(o + (cb > 1 ? (size_t)Tcap : 0));
    c.o_ids = o; o = align16(o + (cb > 1 ? (size_t)cb * 4 : 0));
    c.o_gs = o; o = align16(o + (cb > 1 ? (size_t)(Tcap + 1) * 2 : 0));
    c.o_ring = o; o = align16(o + (cb > 1 ? (size_t)2 * kStageEntries * 8 : 0));
    c.o_tring = o; o = align16(o + (cb > 1 ? (size_t)2 * kTopoEntries * 2 : 0));
    c.o_wm = o; o = align16(o + (cb > 1 ? (size_t)2 * ((Tcap + 63) / 64) * 8 : 0));   // write mask + fire mask words
    c.o_sm1 = c.o_xm1 = c.o_v1 = 0;
    c.bytes = o;
    return c;
}

__device__ __forceinline__ void dd_bind(DD &d, LDS uint8_t *smem, const Scratch &sc, int slot, int cb = 1) {
    LdsCarve c = lds_carve(sc.Tcap, sc.Lcap, cb, sc.us);
    LDS uint32_t *lay = (LDS uint32_t *)(smem + c.o_lay);
    d.noff = lay;
    d.nn = lay + sc.Tcap;
    d.nalive = lay + 2 * sc.Tcap;
    d.aoff = lay + 3 * sc.Tcap;
    d.acnt = lay + 4 * sc.Tcap;
    d.rslot = (LDS int16_t *)(smem + c.o_rslot);
    d.us = sc.us;
    d.buf0 = (LDS double *)(smem + c.o_buf);
    d.buf1 = d.buf0 + kLdsWidth;
    d.coef = (LDS double *)(smem + c.o_coef);
    d.walk = (LDS int16_t *)(smem + c.o_walk);
    d.sm1 = sc.sm1 + (size_t)slot * sc.Tcap;
    d.xm1 = sc.xm1 + (size_t)slot * sc.Tcap;
    d.v1 = sc.v1 + (size_t)slot * sc.Tcap;
    size_t N = (size_t)slot * sc.Ncap, A = (size_t)slot * sc.Acap;
    d.ntopo = sc.ntopo + N;
    d.nflag = sc.nflag + N;
    d.nmask = sc.nmask + N;
    d.outcnt = sc.outcnt + N;
    d.s2 = sc.s2 + N;
    d.tw = sc.tw + N;
    d.atopo = sc.atopo + A;
    d.aflag = sc.aflag + A;
    // no packed-topology mirror unless k_relax's batched path builds one (build_stream): the
    // other kernels (refine, emit, one-cut apply) edit the master flags only
    d.tmir = nullptr;
    d.gstart = nullptr;
    d.stream = 0;
    d.ng = 0;
    d.kg = 0;
    d.Nn = 0;
    d.Amir = 0;
}

// Coefficient slot of state rank r at DD layer k (arc from tree layer k-1 into k).
// Structural layer (decides which decision the rank is) = g+k-1; coefficient layer
// (decides the key's (q, i)) = sol_len+k-1, exactly the reference's running index
// `i` (DD.cpp:3940,3952) -- the two differ only for records whose solution vector
// is shorter than their global layer.
__device__ __forceinline__ int rank_slot(const NetDev &net, const DD &d, int k, int r) {
    int ls = d.g + k - 1;
    if (d.aligned) return net.slot_tab[ls * kMaxU + r];
    int u = net.layer_universe[ls];
    if (u < 0 || r >= net.set_len[u]) return -1;
    int dec = net.set_val[net.set_off[u] + r];
    if (dec < 0) return -1;
    int lc = d.len + k - 1;
    int j = net.arc_head[dec];
    for (int s = net.slot_off[lc]; s < net.slot_off[lc + 1]; s++)
        if (net.slot_head[s] == j) return s;
    return net.n_slots;
}

__device__ __forceinline__ int16_t rank_value(const NetDev &net, int layer, int r) {
    int u = net.layer_universe[layer];
    return net.set_val[net.set_off[u] + r];
}

// Arc weight as the reference stores it: the coefficient of the last swept cut,
// 0 before any cut and always 0 for a -1 decision (DD.cpp:3559-3560, 3866-3868).
__device__ __forceinline__ double arc_weight(const NetDev &net, const DD &d, int k, int r, const GBL double *row) {
    if (!row || r == 0) return 0.0;
    int s = rank_slot(net, d, k, r);
    return s >= 0 ? row[s] : 0.0;
}

// per-layer coefficient table in LDS: coef[r] for every rank
__device__ __forceinline__ void load_layer_coef(const NetDev &net, const DD &d, int k, const GBL double *row) {
    if (lane() < d.us) {
        int s = (lane() == 0) ? -1 : rank_slot(net, d, k, lane());
        d.coef[lane()] = s >= 0 ? row[s] : 0.0;
    }
}

// ------------------------------------------------------------------------------------
// Build (buildTree + buildNextLayer).  Returns false on capacity overflow.
// The state masks of a layer of at most kBuildLds nodes are also kept in LDS (the value
// buffers, unused during the build), so that the next layer reads them without an HBM
// round trip and the layer step waits for no store; wider layers go through HBM.
constexpr uint32_t kBuildLds = (uint32_t)kLdsWidth * 2;   // u32 masks per parity half of buf0/buf1
__device__ __forceinline__ bool dd_build(const NetDev &net, DD &d, const Scratch &sc, uint32_t root_mask, uint32_t &n_nodes,
                         uint32_t &n_arcs, uint32_t &n_merged) {
    const int L = net.L;
    LDS uint32_t *mb = (LDS uint32_t *)d.buf0;     // [2][kBuildLds]
    if (lane() == 0) {
        d.ntopo[0] = kNoRank << kRankShift;
        d.nflag[0] = kAlive | kInAlive;
        d.nmask[0] = root_mask;
        d.s2[0] = DMIN;
        d.noff[0] = 0; d.nn[0] = 1; d.nalive[0] = 1; d.aoff[0] = 0; d.acnt[0] = 0;
        mb[0] = root_mask;
    }
    wave_mem_sync();
    uint32_t total_nodes = 1, total_arcs = 0, merged_nodes = 0;
    uint32_t next_size = 0;
    int idx = 0;
    int exact = 1;
    bool ok = true;
    bool in_lds = true;                            // masks of the current layer in mb[idx & 1]
    for (int a = d.g; a < L; a++, idx++) {
        if (idx + 2 > sc.Tcap) { ok = false; break; }
        const uint32_t cnoff = uni(d.noff[idx]), cn = uni(d.nn[idx]);
        LDS uint32_t *cm = mb + (size_t)(idx & 1) * kBuildLds;        // current layer (LDS copy)
        LDS uint32_t *nm = mb + (size_t)((idx + 1) & 1) * kBuildLds;  // next layer (LDS copy)
        const int upd = net.layer_update[a];
        uint32_t full = 0;
        if (upd >= 0) {  // stateUpdateMap.contains(a): every current-layer node takes the full set
            const int sl = net.set_len[upd];
            full = (sl >= 32) ? 0xFFFFFFFFu : ((1u << sl) - 1u);
            for (uint32_t i = lane(); i < cn; i += kWave) d.nmask[cnoff + i] = full;
            next_size = cn * (uint32_t)sl;
        }
        auto mask_of = [&](uint32_t i) -> uint32_t {
            if (upd >= 0) return full;
            return in_lds ? cm[i] : d.nmask[cnoff + i];
        };
        if (next_size >= kCollapseWidth && (unsigned)(d.g + idx) < net.L5) {
            // collapse into one node; one arc per (parent, state) in order
            exact = 0;
            const uint32_t mnode = total_nodes, base_arc = total_arcs;
            uint32_t carry = 0, uni = 0;
            for (uint32_t base = 0; base < cn; base += kWave) {
                uint32_t i = base + lane();
                bool valid = i < cn;
                uint32_t m = valid ? mask_of(i) : 0u;
                uint32_t c = __popc(m);
                uint32_t incl = wave_scan_incl(c);
                uint32_t off = base_arc + carry + incl - c;
                if (valid && off + c <= (uint32_t)sc.Acap) {
                    uint32_t t = 0, mm = m;
                    while (mm) {
                        uint32_t r = __ffs(mm) - 1;
                        mm &= mm - 1;
                        d.atopo[off + t] = i | (r << kRankShift);
                        d.aflag[off + t] = kAlive;
                        t++;
                    }
                    d.outcnt[cnoff + i] = c;
                }
                uni |= m;
                carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
            }
            uni = wave_or(uni);
            if (base_arc + carry > (uint32_t)sc.Acap || mnode + 1 > (uint32_t)sc.Ncap) { ok = false; break; }
            if (lane() == 0) {
                d.ntopo[mnode] = kNoRank << kRankShift;
                d.nflag[mnode] = kAlive | kInAlive;
                d.nmask[mnode] = uni;
                d.s2[mnode] = DMIN;
                d.noff[idx + 1] = mnode; d.nn[idx + 1] = 1; d.nalive[idx + 1] = 1;
                d.aoff[idx + 1] = base_arc; d.acnt[idx + 1] = carry;
                nm[0] = uni;
            }
            total_nodes += 1;
            merged_nodes += 1;
            total_arcs += carry;
            next_size = __popc(uni);
            in_lds = true;
        } else {
            // exact expansion: one child per (parent, state), child states = parent minus decision
            const uint32_t first = total_nodes;
            uint32_t carry = 0, ns = 0;
            for (uint32_t base = 0; base < cn; base += kWave) {
                uint32_t i = base + lane();
                bool valid = i < cn;
                uint32_t m = valid ? mask_of(i) : 0u;
                uint32_t c = __popc(m);
                uint32_t incl = wave_scan_incl(c);
                uint32_t off = first + carry + incl - c;
                uint32_t has0 = m & 1u;
                uint32_t cs = has0 ? c + (c - 1) * (c - 1) : c * (c ? c - 1 : 0);
                if (valid && off + c <= (uint32_t)sc.Ncap) {
                    uint32_t t = 0, mm = m;
                    while (mm) {
                        uint32_t r = __ffs(mm) - 1;
                        mm &= mm - 1;
                        const uint32_t ch = off + t;
                        const uint32_t cmask = (r == 0) ? m : (m & ~(1u << r));
                        d.ntopo[ch] = i | (r << kRankShift);
                        d.nflag[ch] = kAlive | kInAlive;
                        d.nmask[ch] = cmask;
                        d.s2[ch] = DMIN;
                        if (ch - first < kBuildLds) nm[ch - first] = cmask;
                        t++;
                    }
                    d.outcnt[cnoff + i] = c;
                }
                ns += wave_sum(valid ? cs : 0u);
                carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
            }
            if (first + carry > (uint32_t)sc.Ncap) { ok = false; break; }
            if (lane() == 0) {
                d.noff[idx + 1] = first; d.nn[idx + 1] = carry; d.nalive[idx + 1] = carry;
                d.aoff[idx + 1] = total_arcs; d.acnt[idx + 1] = 0;  // aoff: merged arcs before the layer
            }
            total_nodes += carry;
            next_size = ns;
            in_lds = carry <= kBuildLds;
        }
        // the next layer reads its masks from LDS, or from HBM after the stores completed
        if (in_lds) wave_lds_sync();
        else wave_mem_sync();
    }
    if (!ok) return false;
    d.T = idx + 1;
    d.exact = exact;
    // terminal arcs: weight DOUBLE_MAX (DD.cpp:3587-3597); one out-arc per last-layer node
    const uint32_t lo = uni(d.noff[d.T - 1]), ln = uni(d.nn[d.T - 1]);
    for (uint32_t i = lane(); i < ln; i += kWave) {
        d.tw[lo + i] = DMAX;
        d.outcnt[lo + i] = 1;
    }
    n_nodes = total_nodes + 1;                                            // + terminal
    n_arcs = (total_nodes - 1 - merged_nodes) + total_arcs + ln;          // exact in-arcs + merged + terminal
    n_merged = total_arcs;
    wave_mem_sync();
    return true;
}

// ------------------------------------------------------------------------------------
// One cut sweep over layers 1..T-1 (the shared body of both apply functions).
__device__ __forceinline__ void dd_sweep(const NetDev &net, DD &d, const GBL double *row, double root_value) {
    if (lane() == 0) {
        d.s2[0] = root_value;
        d.buf0[0] = root_value;
    }
    for (int k = lane(); k < d.T; k += kWave) d.v1[k] = 0;
    wave_mem_sync();   // the summaries live in HBM: clear before the sweep sets them
    for (int k = 1; k < d.T; k++) {
        const uint32_t noff = uni(d.noff[k]), n = uni(d.nn[k]);
        const uint32_t pnoff = uni(d.noff[k - 1]), pn = uni(d.nn[k - 1]);
        const bool prev_lds = pn <= (uint32_t)kLdsWidth;
        const bool cur_lds = n <= (uint32_t)kLdsWidth;
        const bool w1 = uni(d.nalive[k]) == 1;
        LDS double *pbuf = (k & 1) ? d.buf0 : d.buf1;
        LDS double *cbuf = (k & 1) ? d.buf1 : d.buf0;
        load_layer_coef(net, d, k, row);
        wave_lds_sync();
        const uint32_t acnt = uni(d.acnt[k]);
        if (acnt) {
            // merged node: max over its alive incoming arcs, in creation order
            const uint32_t aoff = uni(d.aoff[k]);
            VP best{0.0, INT_MIN};
            double xmin = DMAX;
            for (uint32_t base = 0; base < acnt; base += kWave) {
                uint32_t a = base + lane();
                if (a < acnt && (d.aflag[aoff + a] & kAlive)) {
                    uint32_t t = d.atopo[aoff + a];
                    uint32_t p = t & kParentMask, r = t >> kRankShift;
                    double x = prev_lds ? pbuf[p] : d.s2[pnoff + p];
                    VP c;
                    if (r != 0) { c.v = x + d.coef[r]; c.p = prio_new((int)a); xmin = fmin(xmin, c.v); }
                    else { c.v = x; c.p = prio_old((int)a); xmin = fmin(xmin, x + 0.0); }
                    best = vp_pick(best, c);
                }
            }
            best = wave_vp(best);
            xmin = wave_fmin(xmin);
            double v = (best.p == INT_MIN) ? DMIN : smax(best.v, DMIN);
            if (lane() == 0) {
                d.s2[noff] = v;
                cbuf[0] = v;
                if (w1) { d.sm1[k] = v; d.xm1[k] = xmin; d.v1[k] = 1; }
            }
        } else {
            for (uint32_t base = 0; base < n; base += kWave) {
                uint32_t i = base + lane();
                if (i < n) {
                    uint32_t node = noff + i;
                    uint8_t f = d.nflag[node];
                    if (f & kAlive) {
                        uint32_t t = d.ntopo[node];
                        uint32_t p = t & kParentMask, r = t >> kRankShift;
                        double x, y = DMAX;
                        if (!(f & kInAlive)) x = DMIN;
                        else {
                            double px = prev_lds ? pbuf[p] : d.s2[pnoff + p];
                            if (r != 0) { x = px + d.coef[r]; y = x; }
                            else { x = px; y = px + 0.0; }
                        }
                        d.s2[node] = x;
                        if (cur_lds) cbuf[i] = x;
                        if (w1) { d.sm1[k] = x; d.xm1[k] = y; d.v1[k] = 1; }
                    }
                }
            }
        }
        if (!cur_lds || !prev_lds) wave_mem_sync();
        else wave_lds_sync();
    }
    wave_mem_sync();
}

// arg-max with first-wins ties over alive nodes of layer k; value getter by functor
template <typename F>
__device__ __forceinline__ VP layer_max_first(const DD &d, int k, F val) {
    const uint32_t noff = uni(d.noff[k]), n = uni(d.nn[k]);
    VP best{0.0, INT_MIN};
    for (uint32_t base = 0; base < n; base += kWave) {
        uint32_t i = base + lane();
        if (i < n && (d.nflag[noff + i] & kAlive)) best = vp_pick(best, VP{val(noff + i), prio_old((int)i)});
    }
    return wave_vp(best);
}

// the single alive node of a width-1 layer
__device__ __forceinline__ uint32_t layer_single(const DD &d, int k) {
    const uint32_t noff = uni(d.noff[k]), n = uni(d.nn[k]);
    uint32_t found = 0xFFFFFFFFu;
    for (uint32_t base = 0; base < n; base += kWave) {
        uint32_t i = base + lane();
        uint64_t b = __ballot(i < n && (d.nflag[noff + i] & kAlive));
        if (b) { found = noff + base + (uint32_t)(__ffsll((unsigned long long)b) - 1); break; }
    }
    return found;
}

// Exact pruning of one width-1 layer (the body of the loops at DD.cpp:3899-3924 /
// 3991-4016): every alive in-arc with parent.state2 + weight + gain <= thresh goes.
// Returns false when all of them would go (the caller returns false / DOUBLE_MIN).
__device__ __forceinline__ bool dd_prune_layer(const NetDev &net, DD &d, const GBL double *row, int k, double maxState, double thresh) {
    const uint32_t M = layer_single(d, k);
    const double gain = maxState - d.s2[M];
    const uint32_t pnoff = uni(d.noff[k - 1]);
    load_layer_coef(net, d, k, row);
    wave_lds_sync();
    const uint32_t acnt = uni(d.acnt[k]);
    uint32_t total = 0, pruned = 0;
    if (acnt) {
        const uint32_t aoff = uni(d.aoff[k]);
        for (uint32_t base = 0; base < acnt; base += kWave) {
            uint32_t a = base + lane();
            bool alive = a < acnt && (d.aflag[aoff + a] & kAlive);
            bool pr = false;
            if (alive) {
                uint32_t t = d.atopo[aoff + a];
                uint32_t p = t & kParentMask, r = t >> kRankShift;
                double w = (r == 0) ? 0.0 : d.coef[r];
                pr = ((d.s2[pnoff + p] + w) + gain) <= thresh;
                if (pr) {
                    d.aflag[aoff + a] = 0;
                    mir_arc_clear(d, aoff + a);
                    gsub(&d.outcnt[pnoff + p], 1u);
                }
            }
            total += wave_sum(alive ? 1u : 0u);
            pruned += wave_sum(pr ? 1u : 0u);
        }
    } else {
        uint32_t t = d.ntopo[M];
        uint8_t f = d.nflag[M];
        uint32_t p = t & kParentMask, r = t >> kRankShift;
        if (f & kInAlive) {
            total = 1;
            double w = (r == 0) ? 0.0 : d.coef[r];
            if (((d.s2[pnoff + p] + w) + gain) <= thresh) {
                pruned = 1;
                if (lane() == 0) {
                    d.nflag[M] = f & (uint8_t)~kInAlive;
                    mir_node_clear(d, M, kMirIn);
                    d.outcnt[pnoff + p] -= 1u;
                }
            }
        }
    }
    wave_mem_sync();
    return total != pruned;
}

// Does any width-1 layer in [first, end) prune something?  From per-layer summaries:
// rounding is monotone, so some arc satisfies fl(fl(s + w) + gain) <= thresh exactly
// when fl(xmin + gain) <= thresh.  Layers without a summary count as firing.
// Returns a 64-bit mask of firing layers for the 64-layer window starting at `base`.
template <typename PV, typename PF>
__device__ __forceinline__ uint64_t prune_fire(const DD &d, int base, int end, double maxState, double thresh,
                                      PV sm, PV xm, int stride, PF valid) {
    int k = base + lane();
    bool fire = false;
    if (k < end && (d.nalive[k]) == 1) {
        if (!valid[k]) fire = true;
        else fire = (xm[(size_t)k * stride] + (maxState - sm[(size_t)k * stride])) <= thresh;
    }
    return __ballot(fire);
}

// Width-1 arc pruning over layers [first, end) (DD.cpp:3895-3928, 3987-4021), after a
// single-cut sweep (s2 and the sm1/xm1 summaries hold this cut).  Returns false when a
// width-1 layer would lose all of its incoming arcs.
__device__ __forceinline__ bool dd_prune(const NetDev &net, DD &d, const GBL double *row, int first, int end, double thresh,
                         double maxState) {
    wave_mem_sync();   // summaries written by other lanes of the sweep (HBM)
    for (int base = first; base < end; base += kWave) {
        uint64_t b = prune_fire(d, base, end, maxState, thresh, d.sm1, d.xm1, 1, d.v1);
        while (b) {
            int k = base + (int)(__ffsll((unsigned long long)b) - 1);
            b &= b - 1;
            if (!dd_prune_layer(net, d, row, k, maxState, thresh)) return false;
        }
    }
    return true;
}

// Values of the last layer for the cut being post-processed: v(i) = p[i * stride].
struct LastVals {
    const GBL double *p;
    int stride;
    __device__ __forceinline__ double operator()(uint32_t i) const { return p[(size_t)i * stride]; }
};

// Bottom-up deletion cascade (removeNode / bottomUpDelete / updateTree,
// DD.cpp:4040-4153): last-layer nodes marked for removal die, and a parent dies when its
// last alive out-arc dies in this batch.  code = 0: the last layer's marks are kKill;
// code > 0: they are the feasibility scan's first-removing-cut codes (nflag bits 3..7 ==
// code, see f_leaf_scan_t).  Node flags of a layer are read U per lane at a time and the
// parents' out-degree decrements issued together.
__device__ __forceinline__ void dd_cascade(DD &d, uint32_t code) {
    constexpr int U = 4;
    const int last = d.T - 1;
    for (int k = last; k >= 1; k--) {
        const uint32_t noff = uni(d.noff[k]), n = uni(d.nn[k]), pnoff = uni(d.noff[k - 1]);
        const uint32_t acnt = uni(d.acnt[k]);
        uint32_t killed = 0, parent_killed = 0;
        if (acnt) {
            const uint32_t M = noff;
            if (d.nflag[M] & kKill) {
                killed = 1;
                const uint32_t aoff = uni(d.aoff[k]);
                for (uint32_t base = 0; base < acnt; base += kWave) {
                    uint32_t a = base + lane();
                    bool pk = false;
                    if (a < acnt && (d.aflag[aoff + a] & kAlive)) {
                        uint32_t p = d.atopo[aoff + a] & kParentMask;
                        d.aflag[aoff + a] = 0;
                        mir_arc_clear(d, aoff + a);
                        if (gsub(&d.outcnt[pnoff + p], 1u) == 1u) {
                            d.nflag[pnoff + p] |= kKill;
                            pk = true;
                        }
                    }
                    parent_killed += (uint32_t)__popcll(__ballot(pk));
                }
                wave_mem_sync();
                if (lane() == 0) {
                    d.nflag[M] = 0;
                    mir_node_clear(d, M, kMirAlive | kMirIn);
                }
            }
        } else {
            const bool by_code = code != 0 && k == last;
            for (uint32_t base = 0; base < n; base += U * kWave) {
                uint32_t f[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const uint32_t i = base + (uint32_t)u * kWave + lane();
                    f[u] = i < n ? (uint32_t)d.nflag[noff + i] : 0u;
                }
                sched_fence();
                bool kk[U];
                uint32_t p[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const uint32_t i = base + (uint32_t)u * kWave + lane();
                    kk[u] = by_code ? ((f[u] & kAlive) != 0 && (f[u] >> 3) == code) : (f[u] & kKill) != 0;
                    p[u] = (kk[u] && (f[u] & kInAlive)) ? (d.ntopo[noff + (i < n ? i : 0u)] & kParentMask) : 0u;
                }
                uint32_t old[U];
#pragma unroll
                for (int u = 0; u < U; u++)
                    old[u] = (kk[u] && (f[u] & kInAlive)) ? gsub(&d.outcnt[pnoff + p[u]], 1u) : 0u;
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const uint32_t i = base + (uint32_t)u * kWave + lane();
                    if (kk[u]) {
                        d.nflag[noff + i] = 0;
                        mir_node_clear(d, noff + i, kMirAlive | kMirIn);
                    }
                    // exactly one decrement sees 1: that lane marks the parent
                    const bool pk = old[u] == 1u;
                    if (pk) d.nflag[pnoff + p[u]] |= kKill;
                    killed += (uint32_t)__popcll(__ballot(kk[u]));
                    parent_killed += (uint32_t)__popcll(__ballot(pk));
                }
            }
        }
        if (lane() == 0) d.nalive[k] -= killed;
        wave_mem_sync();
        if (!parent_killed) break;
    }
}

// Last-layer removal (state2 < -0.01, DD.cpp:3880-3893) and the bottom-up deletion
// cascade (removeNode / bottomUpDelete / updateTree, DD.cpp:4040-4153).  Returns false
// when every alive last-layer node would go (the reference returns false there).
// maxState = max state2 over the surviving last layer (the value the pruning uses).
constexpr int kUnroll = 4;

__device__ __forceinline__ bool dd_remove_last(DD &d, const LastVals &lv, double &maxState) {
    const int last = d.T - 1;
    const uint32_t lo = uni(d.noff[last]), ln = uni(d.nn[last]);
    uint32_t rm = 0;
    VP mx{0.0, INT_MIN};
    for (uint32_t base = 0; base < ln; base += kUnroll * kWave) {
        uint8_t f[kUnroll];
        double v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            uint32_t i = base + u * kWave + lane();
            f[u] = i < ln ? d.nflag[lo + i] : 0;
            v[u] = i < ln ? lv(i) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            uint32_t i = base + u * kWave + lane();
            if (f[u] & kAlive) {
                if (v[u] < -0.01) {
                    d.nflag[lo + i] = f[u] | kKill;
                    rm++;
                } else {
                    mx = vp_pick(mx, VP{v[u], prio_old((int)i)});
                }
            }
        }
    }
    rm = wave_sum(rm);
    mx = wave_vp(mx);
    maxState = (mx.p == INT_MIN) ? DMIN : smax(DMIN, mx.v);
    if (rm == uni(d.nalive[last])) return false;
    if (rm) {
        wave_mem_sync();
        dd_cascade(d, 0u);
    }
    return true;
}

// Terminal arcs of an optimality cut: weight = min(weight, parent.state2), terminal
// state = max over them (DD.cpp:3975-3984); also maxState over the last layer.
__device__ __forceinline__ double dd_terminal(DD &d, const LastVals &lv, double &maxState) {
    const int last = d.T - 1;
    const uint32_t lo = uni(d.noff[last]), ln = uni(d.nn[last]);
    VP best{0.0, INT_MIN}, mx{0.0, INT_MIN};
    for (uint32_t base = 0; base < ln; base += kUnroll * kWave) {
        uint8_t f[kUnroll];
        double v[kUnroll], w[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            uint32_t i = base + u * kWave + lane();
            f[u] = i < ln ? d.nflag[lo + i] : 0;
            v[u] = i < ln ? lv(i) : 0.0;
            w[u] = i < ln ? d.tw[lo + i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            uint32_t i = base + u * kWave + lane();
            if (f[u] & kAlive) {
                double nw = smin(w[u], v[u]);
                d.tw[lo + i] = nw;
                best = vp_pick(best, VP{nw, prio_old((int)i)});
                mx = vp_pick(mx, VP{v[u], prio_old((int)i)});
            }
        }
    }
    best = wave_vp(best);
    mx = wave_vp(mx);
    wave_mem_sync();
    maxState = (mx.p == INT_MIN) ? DMIN : smax(DMIN, mx.v);
    return (best.p == INT_MIN) ? DMIN : smax(DMIN, best.v);
}

// applyFeasibilityCut after a single-cut sweep.
__device__ __forceinline__ bool dd_post_feasibility(const NetDev &net, DD &d, const GBL double *row) {
    double maxState;
    if (!dd_remove_last(d, LastVals{d.s2 + uni(d.noff[d.T - 1]), 1}, maxState)) return false;
    if (!d.exact) return dd_prune(net, d, row, 1, d.T - 1, -0.01, maxState);
    return true;
}

// applyOptimalityCut after a single-cut sweep.  Returns the terminal state (or DOUBLE_MIN).
__device__ __forceinline__ double dd_post_optimality(const NetDev &net, DD &d, const GBL double *row, double optimal) {
    const int last = d.T - 1;
    double maxState;
    const double term = dd_terminal(d, LastVals{d.s2 + uni(d.noff[last]), 1}, maxState);
    if (term <= optimal) return term;
    if (!d.exact) {
        if (!dd_prune(net, d, row, 3, last - 1, optimal - 0.01, maxState)) return DMIN;
    }
    return term;
}

// ------------------------------------------------------------------------------------
// Multi-cut sweeps.  Deleting nodes never changes state2 of the nodes that stay (an
// alive node keeps every non-pruned in-arc and the tails of those arcs stay alive), so
// the sweeps of CB consecutive pool cuts of one type can run together over the same DD
// and their removal / terminal / early-exit logic be replayed in pool order afterwards.
// Only width-1 arc pruning changes later sweeps: per (width-1 layer, cut) the sweep
// records the single node's state2 and the smallest parent.state2 + weight over its
// in-arcs; since rounding is monotone, "some arc is pruned" <=> fl(xmin + gain) <=
// threshold.  When that fires (or deletions make a new width-1 layer) the cut is redone
// with the exact single-cut path and the batch restarts after it.
//
// Layout during a batch: the narrow layers (< 128 nodes: every layer but the last
// few) keep their CB values per node in LDS, and their packed 16-bit topology words and
// coefficients are staged into LDS rings a group of layers ahead, so that a layer step
// waits on no HBM load; the wide tail layers stream through HBM (s2b, CB values per
// node); for optimality batches the last layer is never materialised: two fused passes
// compute the leaf values on the fly.

struct BatchView {
    LDS double *vb;        // [2][kLdsBatchWidth][CB]
    LDS double *cring;     // [2][kStageEntries] staged coefficients of the narrow layers
    LDS uint16_t *tring;   // [2][kTopoEntries] staged topology words of the narrow layers
    LDS double *coef;      // [CB][ustride]
    LDS uint8_t *w1;       // [Tcap]: layer had one alive node when the batch started
    LDS int32_t *ids;      // [CB]: pool row of each batch cut
    LDS uint64_t *wm;      // [ceil(Tcap/64)] layers whose state2 a sweep writes (exact redo), or null
    LDS uint64_t *fm;      // [ceil(Tcap/64)] width-1 layers whose pruning fires (exact redo)
    const LDS uint64_t *wsel;   // the write mask in force (null: the kS rule)
    GBL double *s2b;       // HBM [tail_cap][CB]: layers >= kg
    GBL double *sm, *xm;   // HBM [Tcap][CB]
    uint32_t gbase;    // noff[kg]
#ifdef SGUFP_PROF
    uint64_t prof[2];  // ticks: coefficient staging, merged layers
#endif
#ifdef SGUFP_TRACE
    int trace_on;
#endif
};


// Packed topology of the narrow layers (see mir_node_clear) and the staging groups of
// the narrow sweep: runs of at most kStageLayers layers whose words fit one topology ring
// slot and whose coefficients (per_layer_max per layer) fit one coefficient ring slot.
// A single layer larger than a slot (a merged layer with > kTopoEntries in-arcs) leaves
// d.stream = 0 and the DD takes the single-cut path.
__device__ __forceinline__ void build_stream(DD &d, uint32_t n_merged_arcs, int per_layer_max) {
    int kg = d.T - 1;
    for (int base = 0; base < d.T - 1; base += kWave) {
        int k = base + lane();
        uint64_t b = __ballot(k < d.T - 1 && (d.nn[k]) > kNarrowMax);
        if (b) { kg = base + (int)(__ffsll((unsigned long long)b) - 1); break; }
    }
    d.kg = kg;
    d.Nn = uni(d.noff[kg]);
    d.Amir = n_merged_arcs;
    d.stream = 0;
    const int maxl = min(kStageLayers, max(1, kStageEntries / max(1, per_layer_max)));
    int ng = 0;
    for (int k = 1; k < kg;) {
        if (lane() == 0) d.gstart[ng] = (uint16_t)k;
        ng++;
        const uint32_t n0 = uni(d.noff[k]), a0 = uni(d.aoff[k]);
        if ((uni(d.noff[k + 1]) - n0) + (uni(d.aoff[k + 1]) - a0) > (uint32_t)kTopoEntries) return;
        int k1 = k + 1;
        while (k1 < kg && k1 - k < maxl &&
               (uni(d.noff[k1 + 1]) - n0) + (uni(d.aoff[k1 + 1]) - a0) <= (uint32_t)kTopoEntries)
            k1++;
        k = k1;
    }
    if (lane() == 0) d.gstart[ng] = (uint16_t)kg;
    d.ng = ng;
    d.stream = 1;
    for (uint32_t i = lane(); i < d.Nn; i += kWave) {
        uint32_t t = d.ntopo[i];
        uint8_t f = d.nflag[i];
        d.tmir[i] = (uint16_t)((t & kMirParent) | (((t >> kRankShift) & 31u) << kMirRankShift) |
                               ((f & kAlive) ? kMirAlive : 0) | ((f & kInAlive) ? kMirIn : 0));
    }
    for (uint32_t a = lane(); a < d.Amir; a += kWave) {
        uint32_t t = d.atopo[a];
        // a dead merged arc points at the NaN sentinel slot (see sweep_narrow)
        const bool al = (d.aflag[a] & kAlive) != 0;
        d.tmir[d.Nn + a] = (uint16_t)((al ? (t & kMirParent) : kNarrowMax) | (((t >> kRankShift) & 31u) << kMirRankShift) |
                                      (al ? kMirAlive : 0));
    }
    wave_mem_sync();
}

// coefficients of DD layer k for the batch cuts: bv.coef[c][r] (one load per entry)
__device__ __forceinline__ void batch_coef_direct(const NetDev &net, const DD &d, BatchView &bv, const Pool &pool, int k,
                                         int nb) {
    const int us = pool.ustride, ls = d.g + k - 1;
    const size_t ltab = (size_t)net.L * us;
    for (int idx = lane(); idx < nb * us; idx += kWave) {
        int cc = idx / us, r = idx - cc * us;
        bv.coef[idx] = pool.coefT[(size_t)bv.ids[cc] * ltab + (size_t)ls * us + r];
    }
    wave_lds_sync();
}

// Narrow layers 1 .. kg-1: values in LDS; topology words and coefficients staged into
// LDS rings one group of layers ahead (the loads of group j+1 are issued when group j
// starts, so their latency hides behind the group's layers).
// s2 (single values of the batch's last cut, read later by path walks) is written for
// layers < kS only: the cutset layer can only move up, and exact-layer steps of a walk
// read no state2.
template <int CB>
__device__ __forceinline__ void sweep_narrow(const NetDev &net, DD &d, BatchView &bv, const Pool &pool, int nb,
                                             double rv, int kS, int kend = INT_MAX) {
    constexpr int G = kWave / CB;
    constexpr int PC = kStageEntries / kWave, PT = kTopoEntries / kWave;
    const int c = lane() % CB, grp = lane() / CB;
    const bool cv = c < nb;
    const int us = pool.ustride;
    const int per_layer = nb * us;
    const size_t ltab = (size_t)net.L * us;
    if (lane() < CB && cv) {
        bv.vb[c] = rv;
        if (c == nb - 1) d.s2[0] = rv;
    }
    // NaN sentinel in slot kNarrowMax of both value buffers (dead merged arcs point there)
    if (lane() < 2 * CB)
        bv.vb[(size_t)(lane() / CB) * kLdsBatchWidth * CB + kNarrowMax * CB + (lane() % CB)] = __builtin_nan("");
    if (d.ng == 0) return;
    double pf[PC] = {};
    uint32_t pt[PT] = {};
    auto commit = [&](int slot) {
        LDS double *ring = bv.cring + (size_t)slot * kStageEntries;
        LDS uint16_t *tr = bv.tring + (size_t)slot * kTopoEntries;
#pragma unroll
        for (int jj = 0; jj < PC; jj++) ring[lane() + jj * kWave] = pf[jj];
#pragma unroll
        for (int jj = 0; jj < PT; jj++) tr[lane() + jj * kWave] = (uint16_t)pt[jj];
    };
    // Per-group layer metadata in registers: lane l <-> layer k0 + l of the current staging
    // group (and the layers after it): node offset, merged-arc offset and a packed word
    // nn:8 | acnt:12 | w1 (bit 31), read per layer with v_readlane instead of a serialised
    // LDS round trip per field; mmask: which of those layers are merged layers.
    uint32_t m_noff = 0, m_aoff = 0, m_pk = 0;
    uint64_t mmask = 0;
    // bit 30 of the packed word: this layer's state2 (of the last batch cut) is written --
    // what a path walk reads (merged layers and their parents, above the cutset layer kS)
    // or, in an exact redo, the layers of the write mask
    auto load_meta = [&](int kw) {
        const int k = kw + lane();
        const bool ok = k < d.T;
        const int kk = ok ? k : 0;
        const uint32_t no = d.noff[kk], ao = d.aoff[kk], nn = d.nn[kk], ac = d.acnt[kk];
        const uint32_t an = kk + 1 < d.T ? d.acnt[kk + 1] : 0u;
        const uint32_t w = bv.w1[kk];
        const uint64_t wsw = bv.wsel ? bv.wsel[kk >> 6] : 0ull;
        sched_fence();
        m_noff = no;
        m_aoff = ao;
        const bool wrl = bv.wsel ? ((wsw >> (kk & 63)) & 1ull) != 0 : (k < kS && (kS >= d.T || ac != 0 || an != 0));
        m_pk = (nn < 255u ? nn : 255u) | ((ac & 0xFFFu) << 8) | (wrl ? 0x40000000u : 0u) | (w ? 0x80000000u : 0u);
        mmask = __ballot(ok && ac != 0);
    };
    auto rl = [](uint32_t v, int l) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); };

    // ring entry e = lane + jj * 64 of a group stages the coefficient of layer k0 + lo, batch
    // cut cc, rank r: the per-lane constants are computed once per sweep
    int c_lo[PC];
    uint32_t c_off[PC];
#pragma unroll
    for (int jj = 0; jj < PC; jj++) {
        const int e = lane() + jj * kWave;
        const int lo = e / per_layer, rem = e - lo * per_layer;
        const int cc = rem / us, r = rem - cc * us;
        c_lo[jj] = lo;
        c_off[jj] = (uint32_t)(bv.ids[cc < nb ? cc : 0] * (int)ltab + r);
    }
    // prefetch of the group [k0g, k1g) into registers (layer offsets from the metadata
    // window, which holds both ends)
    auto issue = [&](int k0g, int k1g, int lw0) {
        const uint32_t n0 = rl(m_noff, k0g - lw0), nN = rl(m_noff, k1g - lw0) - n0;
        const uint32_t a0 = rl(m_aoff, k0g - lw0), nA = rl(m_aoff, k1g - lw0) - a0;
        // entries past the group load the group's last layer again (never read): no branch
#pragma unroll
        for (int jj = 0; jj < PC; jj++) {
            const int k = min(k0g + c_lo[jj], k1g - 1);
            pf[jj] = pool.coefT[(size_t)c_off[jj] + (size_t)(uint32_t)((d.g + k - 1) * us)];
        }
#pragma unroll
        for (int jj = 0; jj < PT; jj++) {
            const uint32_t e = (uint32_t)(lane() + jj * kWave);
            const uint32_t idx = e < nN ? n0 + e : (e < nN + nA ? d.Nn + a0 + (e - nN) : 0u);
            pt[jj] = d.tmir[idx];
        }
    };

    // Exact run [ka, kb] of odd depth D (see the call site).  Every node has one in-arc, so
    // a node's value is the fold of its ancestors' steps from layer ka - 1,
    // x = !in ? DMIN : (reg ? x + coef : x) -- the same operations in the same order as
    // layer by layer.  Lanes are (node of layer kb, cut) pairs: item i = pass * G + grp,
    // cut c.  A lane walks up its node's ancestors' topology words (one dependent LDS read
    // per level, batched over the lane's U items), then loads the root value and the
    // coefficients of every level in one batch and folds.  Only layer kb goes through LDS;
    // odd depth puts layers ka - 1 and kb in different value buffers, so items write their
    // results as they go.  Every alive node of the run is an ancestor of an alive node of
    // layer kb (the deletion cascade removes childless parents), so the width-1 summaries
    // and walk state2 of the inner layers are written on the way (lanes that share an
    // ancestor write the same value; items past the layer repeat its last node).
    auto fold_run = [&](auto Dc, int ka, int slot_, int k0_, int kw_, uint32_t gn0_) {
        constexpr int D = decltype(Dc)::value;
        const int kb = ka + D - 1;
        const LDS uint16_t *tr = bv.tring + (size_t)slot_ * kTopoEntries;
        const LDS double *ring_c = bv.cring + (size_t)slot_ * kStageEntries + c * us;
        const LDS double *pb = bv.vb + (size_t)((ka - 1) & 1) * kLdsBatchWidth * CB;
        LDS double *ob = bv.vb + (size_t)(kb & 1) * kLdsBatchWidth * CB;
        const int l0 = ka - k0_, lw = ka - kw_;   // ring / metadata-window positions
        uint32_t ebase[D], nofs[D];
        bool w1s[D], wrs[D];
#pragma unroll
        for (int s = 0; s < D; s++) {
            nofs[s] = rl(m_noff, lw + s);
            ebase[s] = nofs[s] - gn0_;
            w1s[s] = (rl(m_pk, lw + s) >> 31) != 0;
            wrs[s] = ((rl(m_pk, lw + s) >> 30) & 1u) != 0;
        }
        const uint32_t nlast = rl(m_pk, lw + D - 1) & 255u;
        const bool wlane = c == nb - 1;   // the lane whose cut's state2 the path walks read
        auto items = [&](auto Uc, uint32_t base) {
            constexpr int U = decltype(Uc)::value;
            uint32_t cur[U], wl[U][D];   // wl: topology word | node index << 16, per level
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t i = base + (uint32_t)(u * G + grp);
                cur[u] = i < nlast ? i : nlast - 1u;
            }
#pragma unroll
            for (int s = D - 1; s >= 0; s--) {
                uint32_t w[U];
#pragma unroll
                for (int u = 0; u < U; u++) w[u] = (uint32_t)tr[ebase[s] + cur[u]];
                sched_fence();
#pragma unroll
                for (int u = 0; u < U; u++) {
                    wl[u][s] = w[u] | (cur[u] << 16);
                    cur[u] = mir_parent(w[u]);
                }
            }
            double x[U], cf[U][D];
#pragma unroll
            for (int u = 0; u < U; u++) {
                x[u] = pb[cur[u] * CB + c];
#pragma unroll
                for (int s = 0; s < D; s++)
                    cf[u][s] = ring_c[(size_t)(l0 + s) * per_layer + mir_rank(wl[u][s])];
            }
            sched_fence();
#pragma unroll
            for (int u = 0; u < U; u++) {
                const bool alive = (wl[u][D - 1] & kMirAlive) != 0;
                double xv = x[u], xs[D], xms[D];
#pragma unroll
                for (int s = 0; s < D; s++) {
                    const uint32_t w = wl[u][s];
                    const bool in = (w & kMirIn) != 0, reg = (w & (31u << kMirRankShift)) != 0;
                    const double xn = !in ? DMIN : (reg ? xv + cf[u][s] : xv);
                    xms[s] = !in ? DMAX : (reg ? xn : xv + 0.0);
                    xs[s] = xv = xn;
                }
                ob[(wl[u][D - 1] >> 16) * CB + c] = xv;
                // the summaries / walk values of the run's layers: one divergent branch per
                // item (the per-layer conditions are wave-uniform)
                if (alive && cv) {
#pragma unroll
                    for (int s = 0; s < D; s++) {
                        if (w1s[s]) {
                            bv.sm[(size_t)(ka + s) * CB + c] = xs[s];
                            bv.xm[(size_t)(ka + s) * CB + c] = xms[s];
                        }
                    }
                    if (wlane) {
#pragma unroll
                        for (int s = 0; s < D; s++)
                            if (wrs[s]) d.s2[nofs[s] + (wl[u][s] >> 16)] = xs[s];
                    }
                }
            }
        };
        const uint32_t per = (nlast + G - 1) / G;
        if (per <= 1) items(std::integral_constant<int, 1>{}, 0u);
        else
            for (uint32_t base = 0; base < nlast; base += 2 * G) items(std::integral_constant<int, 2>{}, base);
    };

    // the metadata window (base kw) is reloaded only when the next group's prefetch would
    // leave it (groups are a few layers, the window 64)
    int j = 0, slot = 0;
    int k0 = uni((int)d.gstart[0]), k1 = uni((int)d.gstart[1]);
    int kw = k0;
    load_meta(kw);
    issue(k0, k1, kw);
    commit(0);
    if (d.ng > 1) issue(k1, uni((int)d.gstart[2]), kw);
    uint32_t gn0 = rl(m_noff, 0), gnN = rl(m_noff, k1 - kw) - gn0, ga0 = rl(m_aoff, 0);
    wave_lds_sync();
    const int ke = min(d.kg, kend);   // layers >= kend are not needed (exact redo)
    for (int k = 1; k < ke;) {
        if (k == k1) {
#ifdef SGUFP_PROF
            const uint64_t t_sw = wall_clock64();
#endif
            // next group: its words and coefficients were issued one group ago
            j++;
            slot ^= 1;
            commit(slot);
#ifdef SGUFP_PROF_COMMIT
            bv.prof[1] += wall_clock64() - t_sw;
#endif
            k0 = k1;
            k1 = uni((int)d.gstart[j + 1]);
            const int k2 = j + 1 < d.ng ? uni((int)d.gstart[j + 2]) : k1;
            if (k2 - kw >= kWave) {
                kw = k0;
                load_meta(kw);
            }
            if (j + 1 < d.ng) issue(k1, k2, kw);
            gn0 = rl(m_noff, k0 - kw);
            gnN = rl(m_noff, k1 - kw) - gn0;
            ga0 = rl(m_aoff, k0 - kw);
            wave_lds_sync();
#ifdef SGUFP_PROF
            bv.prof[0] += wall_clock64() - t_sw;
#endif
        }
        const int l = k - k0, lm = k - kw;
        const LDS double *coefk = bv.cring + (size_t)slot * kStageEntries + (size_t)l * per_layer;
        const LDS uint16_t *tr = bv.tring + (size_t)slot * kTopoEntries;
        const uint32_t pk = rl(m_pk, lm);
        const uint32_t noff = rl(m_noff, lm), acnt = (pk >> 8) & 0xFFFu;
        const LDS double *pbuf = bv.vb + (size_t)((k - 1) & 1) * kLdsBatchWidth * CB;
        LDS double *cbuf = bv.vb + (size_t)(k & 1) * kLdsBatchWidth * CB;
        const bool w1 = (pk >> 31) != 0;
        if (acnt) {
#ifdef SGUFP_PROF
            const uint64_t t_m = wall_clock64();
#endif
            // state2 of the last batch cut: only what a path walk reads (merged nodes and
            // their parents) unless every layer is asked for (kS = T: the exact redo)
            const bool wr = ((pk >> 30) & 1u) != 0;
            const uint32_t aoff = rl(m_aoff, lm);
            const uint32_t ebase = gnN + (aoff - ga0);   // ring entry of the layer's first arc
            auto word = [&](uint32_t e) -> uint32_t { return (uint32_t)tr[e]; };
            // U independent items per lane per step (U sized to the layer): all topology
            // words first, then all parent values / coefficients, so one step costs two LDS
            // round trips and a narrow layer runs no idle unrolled items.
            // Full steps (every item inside the layer) index the ring with immediate offsets;
            // only the last step clamps.
            auto dispatch = [&](uint32_t count, auto &&step) {
                uint32_t base = 0;
                for (; count - base > (uint32_t)G * 8; base += G * 8)
                    step(std::integral_constant<int, 8>{}, std::false_type{}, base);
                const uint32_t per = (count - base + G - 1) / G;
                if (per <= 1) step(std::integral_constant<int, 1>{}, std::true_type{}, base);
                else if (per <= 2) step(std::integral_constant<int, 2>{}, std::true_type{}, base);
                else if (per <= 4) step(std::integral_constant<int, 4>{}, std::true_type{}, base);
                else step(std::integral_constant<int, 8>{}, std::true_type{}, base);
            };
            // Fast path: a plain max / min over the candidates parent + coefficient.  Dead
            // arcs carry parent slot 127 (kNarrowMax), whose value is a quiet NaN that
            // fmax / fmin skip; items past the layer repeat its last arc; the decision -1
            // (rank 0) has coefficient +0.0, so its candidate is parent + 0.0, which is what
            // the width-1 summary takes and equals the parent except for the sign of zero.
            // The (value, priority) pick of the reference's mixed-order folds differs from
            // the plain max only when the maximum is a zero; that case re-runs the layer
            // with the exact pick below.
            double mx = -INFINITY, xmin = INFINITY;
            const uint32_t alast = acnt - 1u;
            const LDS double *pbc = pbuf + c, *cfc = coefk + c * us;
            dispatch(acnt, [&](auto Uc, auto Cc, uint32_t base) {
                constexpr int U = decltype(Uc)::value;
                constexpr bool CLAMP = decltype(Cc)::value;
                uint32_t wd[U];
                const LDS uint16_t *tw = tr + ebase + base + grp;
#pragma unroll
                for (int u = 0; u < U; u++) {
                    if (CLAMP) {
                        const uint32_t a = base + (uint32_t)(u * G + grp);
                        wd[u] = word(ebase + (a < alast ? a : alast));
                    } else {
                        wd[u] = (uint32_t)tw[u * G];
                    }
                }
                sched_fence();
                double px[U], cf[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    px[u] = pbc[mir_parent(wd[u]) * CB];
                    cf[u] = cfc[mir_rank(wd[u])];
                }
                sched_fence();
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const double v = px[u] + cf[u];
                    mx = __builtin_fmax(mx, v);
                    xmin = __builtin_fmin(xmin, v);
                }
            });
            mx = lane_reduce<CB>(mx, [](double a, double b) { return (b > a) ? b : a; });
            // across the lane groups of each cut (lanes that differ in bits >= log2(CB))
            xmin = lane_reduce<CB>(xmin, [](double a, double b) { return __builtin_fmin(a, b); });
            const bool any = mx != -INFINITY;
            VP best{mx, any ? 0 : INT_MIN};
            if (__ballot(mx == 0.0) != 0) {
                best = VP{0.0, INT_MIN};
                dispatch(acnt, [&](auto Uc, auto, uint32_t base) {
                    constexpr int U = decltype(Uc)::value;
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const uint32_t a = base + u * G + grp;
                        const bool ok = (a < acnt) & cv;
                        const uint32_t wd = word(ebase + (ok ? a : 0u));
                        const uint32_t pp = wd & kMirParent, rr = (wd >> kMirRankShift) & 31u;
                        const bool alive = ok & ((wd & kMirAlive) != 0);
                        const double px = pbuf[(alive ? pp : 0u) * CB + c];
                        const double cf = coefk[(alive ? c * us + rr : 0u)];
                        const bool reg = rr != 0;
                        VP e;
                        e.v = reg ? px + cf : px;
                        e.p = alive ? (reg ? prio_new((int)a) : prio_old((int)a)) : INT_MIN;
                        best = vp_pick(best, e);
                    }
                });
                best = wave_vp<CB>(best);
            }
            if (grp == 0 && cv) {
                double v = (best.p == INT_MIN) ? DMIN : smax(best.v, DMIN);
                cbuf[c] = v;
                if (wr && c == nb - 1) d.s2[noff] = v;
                if (w1) {
                    bv.sm[(size_t)k * CB + c] = v;
                    bv.xm[(size_t)k * CB + c] = any ? xmin : DMAX;
                }
            }
            wave_lds_sync();
#ifdef SGUFP_PROF
            bv.prof[1] += wall_clock64() - t_m;
#endif
            k++;
            continue;
        }
        // A run of exact (tree) layers [k, kb] inside the staging group, ended by the next
        // merged layer; odd depth (see fold_run).
        int kb = min(min(k1, ke) - 1, k + kMaxRun - 1);
        {
            const int span = kb - k + 1;
            const uint64_t b = (mmask >> lm) & ((1ull << span) - 1ull);
            if (b) kb = k + (int)(__ffsll((unsigned long long)b) - 1) - 1;
            if (((kb - k) & 1) != 0) kb--;
        }
        switch (kb - k) {
            case 0: fold_run(std::integral_constant<int, 1>{}, k, slot, k0, kw, gn0); break;
            case 2: fold_run(std::integral_constant<int, 3>{}, k, slot, k0, kw, gn0); break;
            default: fold_run(std::integral_constant<int, 5>{}, k, slot, k0, kw, gn0); break;
        }
        wave_lds_sync();
        k = kb + 1;
    }
#ifdef SGUFP_TRACE
    bv.trace_on = 0;
#endif
}

// value of node p of layer k for batch cut c (LDS for narrow layers, HBM for the tail)
template <int CB>
__device__ __forceinline__ double batch_value(const DD &d, const BatchView &bv, int k, uint32_t p, int c) {
    if (k >= d.kg) return bv.s2b[(size_t)(uni(d.noff[k]) + p - bv.gbase) * CB + c];
    return bv.vb[(size_t)(k & 1) * kLdsBatchWidth * CB + p * CB + c];
}

// Values of the layer before a wide layer: node p, all CB batch cuts (32 contiguous
// bytes at CB = 4).  In LDS when that layer is narrow (k - 1 < kg), else in HBM (s2b).
template <int CB, bool PV_LDS>
struct ParentVals {
    const LDS double *lds;
    const GBL double *gbl;
    __device__ __forceinline__ void load(uint32_t p, double (&x)[CB]) const {
#pragma unroll
        for (int c = 0; c < CB; c++) x[c] = PV_LDS ? lds[p * CB + c] : gbl[(size_t)p * CB + c];
    }
};
template <int CB, bool PV_LDS>
__device__ __forceinline__ ParentVals<CB, PV_LDS> parent_vals(const DD &d, const BatchView &bv, int k) {
    ParentVals<CB, PV_LDS> pv;
    pv.lds = bv.vb + (size_t)(k & 1) * kLdsBatchWidth * CB;
    pv.gbl = PV_LDS ? nullptr : bv.s2b + (size_t)(uni(d.noff[k]) - bv.gbase) * CB;
    return pv;
}

// Wide layers (k >= kg) stream through HBM: one node per lane per item, U items per lane
// per step, the CB cut values of a node in registers.  Software pipeline: the topology
// words of step s + 1 are in flight while step s loads its parent values, and the parent
// values of step s + 1 while step s computes (loads issued back to back, fenced).
template <int CB>
struct WideTopo {
    static constexpr int U = CB >= 8 ? 1 : 16 / CB;
    uint32_t t[U], f[U];
};

template <int CB, bool PV_LDS>
__device__ __forceinline__ void sweep_tail_layer_t(const NetDev &net, DD &d, BatchView &bv, const Pool &pool, int k, int nb,
                                                   int kS) {
    constexpr int U = WideTopo<CB>::U;
    constexpr uint32_t STEP = (uint32_t)U * kWave;
    batch_coef_direct(net, d, bv, pool, k, nb);
    const int us = pool.ustride;
    const uint32_t noff = uni(d.noff[k]), n = uni(d.nn[k]);
    // state2 of tail layers is read only by the exact redo (its write mask, or kS = T)
    const bool w1 = uni(bv.w1[k]) != 0;
    const bool wr = bv.wsel ? ((bv.wsel[k >> 6] >> (k & 63)) & 1ull) != 0 : kS >= d.T;
    const ParentVals<CB, PV_LDS> pv = parent_vals<CB, PV_LDS>(d, bv, k - 1);
    GBL double *out = bv.s2b + (size_t)(noff - bv.gbase) * CB;
    auto load_topo = [&](uint32_t base, WideTopo<CB> &tp) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + (uint32_t)u * kWave + lane();
            const uint32_t ic = i < n ? i : 0u;
            tp.t[u] = d.ntopo[noff + ic];
            tp.f[u] = i < n ? (uint32_t)d.nflag[noff + ic] : 0u;
        }
    };
    auto load_px = [&](const WideTopo<CB> &tp, double (&px)[U][CB]) {
#pragma unroll
        for (int u = 0; u < U; u++) pv.load((tp.f[u] & kAlive) ? (tp.t[u] & kParentMask) : 0u, px[u]);
    };
    WideTopo<CB> ta, tb;
    double pxa[U][CB];
    load_topo(0, ta);
    load_px(ta, pxa);
    load_topo(STEP, tb);
    for (uint32_t base = 0; base < n; base += STEP) {
        double pxb[U][CB];
        load_px(tb, pxb);
        WideTopo<CB> tn;
        load_topo(base + 2 * STEP, tn);
        double cf[U][CB];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int c = 0; c < CB; c++) cf[u][c] = bv.coef[c * us + (ta.t[u] >> kRankShift)];
        sched_fence();
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + (uint32_t)u * kWave + lane();
            if (!(ta.f[u] & kAlive)) continue;
            const uint32_t r = ta.t[u] >> kRankShift;
            const bool inal = (ta.f[u] & kInAlive) != 0;
            double x[CB];
#pragma unroll
            for (int c = 0; c < CB; c++) {
                x[c] = !inal ? DMIN : (r != 0 ? pxa[u][c] + cf[u][c] : pxa[u][c]);
                out[(size_t)i * CB + c] = x[c];
            }
            if (wr) {
                double v = x[0];
#pragma unroll
                for (int c = 1; c < CB; c++) v = (c == nb - 1) ? x[c] : v;
                d.s2[noff + i] = v;
            }
            if (w1) {
#pragma unroll
                for (int c = 0; c < CB; c++) {
                    if (c < nb) {
                        bv.sm[(size_t)k * CB + c] = x[c];
                        bv.xm[(size_t)k * CB + c] = !inal ? DMAX : (r != 0 ? x[c] : pxa[u][c] + 0.0);
                    }
                }
            }
        }
        ta = tb;
        tb = tn;
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int c = 0; c < CB; c++) pxa[u][c] = pxb[u][c];
    }
    wave_mem_sync();
}

template <int CB>
__device__ __forceinline__ void sweep_tail_layer(const NetDev &net, DD &d, BatchView &bv, const Pool &pool, int k, int nb,
                                                 int kS) {
    if (k - 1 < d.kg) sweep_tail_layer_t<CB, true>(net, d, bv, pool, k, nb, kS);
    else sweep_tail_layer_t<CB, false>(net, d, bv, pool, k, nb, kS);
}

// Pruning test of the batch cuts c0 .. c1-1 from the batch summaries over layers
// [first, end): bit c set = redo cut c exactly (some arc is pruned, or a width-1 layer
// has no summary because deletions made it width-1 inside the batch).  The summary loads
// of two 64-layer windows are issued together, independent of the layer flags.
template <int CB>
__device__ __forceinline__ uint32_t dd_prune_mask(const DD &d, const BatchView &bv, int c0, int c1, int first, int end,
                                                  double thresh, const double (&maxState)[CB]) {
    constexpr int W = 2;
    uint32_t mask = 0;
    for (int base = first; base < end; base += W * kWave) {
        bool need[W], val[W];
        double sm[W][CB], xm[W][CB];
#pragma unroll
        for (int w = 0; w < W; w++) {
            const int k = base + w * kWave + lane();
            const int kk = k < end ? k : first;
            need[w] = k < end && d.nalive[kk] == 1;
            val[w] = bv.w1[kk] != 0;
#pragma unroll
            for (int c = 0; c < CB; c++) {
                sm[w][c] = bv.sm[(size_t)kk * CB + c];
                xm[w][c] = bv.xm[(size_t)kk * CB + c];
            }
        }
        sched_fence();
#pragma unroll
        for (int c = 0; c < CB; c++) {
            if (c < c0 || c >= c1) continue;
            bool fire = false;
#pragma unroll
            for (int w = 0; w < W; w++) fire |= need[w] && (!val[w] || (xm[w][c] + (maxState[c] - sm[w][c])) <= thresh);
            if (__ballot(fire)) mask |= 1u << c;
        }
    }
    return mask;
}

template <int CB>
__device__ __forceinline__ bool dd_prune_check(const DD &d, const BatchView &bv, int c, int first, int end, double thresh,
                               double maxState) {
    double ms[CB];
#pragma unroll
    for (int cc = 0; cc < CB; cc++) ms[cc] = maxState;
    return dd_prune_mask<CB>(d, bv, c, c + 1, first, end, thresh, ms) != 0;
}

// Fused last layer of an optimality batch (leaf value = parent value + coefficient).
// Pass A: per cut the terminal state after the running-min update and maxState; it
// commits the terminal weights of all nb cuts (the common case) and keeps the previous
// weights in `keep`.  Pass B, only when the replay stops inside the batch: the weights of
// cuts 0 .. capply from the kept ones.  Streaming as in sweep_tail_layer_t.  The maxima
// are plain maxima; the (value, priority) pick of the reference's ordered folds differs
// from them only when a maximum is a zero, and then fused_leaf_pick recomputes that cut's
// pick exactly.
template <int CB, bool PV_LDS>
__device__ __forceinline__ void fused_leaf_pick(const DD &d, const BatchView &bv, const Pool &pool, int ncut, const GBL double *keep,
                                             int cc, VP &term, VP &mxs) {
    const int last = d.T - 1;
    const uint32_t lo = uni(d.noff[last]), ln = uni(d.nn[last]);
    const int us = pool.ustride;
    const ParentVals<CB, PV_LDS> pv = parent_vals<CB, PV_LDS>(d, bv, last - 1);
    term = VP{0.0, INT_MIN};
    mxs = VP{0.0, INT_MIN};
    for (uint32_t i = lane(); i < ln; i += kWave) {
        const uint32_t f = d.nflag[lo + i];
        if (!(f & kAlive)) continue;
        const uint32_t t = d.ntopo[lo + i], r = t >> kRankShift;
        const bool inal = (f & kInAlive) != 0;
        double px[CB];
        pv.load(t & kParentMask, px);
        double ww = keep[(size_t)i * CB], v = 0.0;
        for (int c = 0; c <= cc; c++) {
            v = !inal ? DMIN : (r != 0 ? px[c] + bv.coef[c * us + r] : px[c]);
            const double nw = smin(ww, v);
            if (c < ncut) ww = nw;
        }
        term = vp_pick(term, VP{ww, prio_old((int)i)});
        mxs = vp_pick(mxs, VP{v, prio_old((int)i)});
    }
    term = wave_vp(term);
    mxs = wave_vp(mxs);
}

template <int CB, bool PASS_A, bool PV_LDS>
__device__ __forceinline__ void fused_leaf_t(const DD &d, BatchView &bv, const Pool &pool, int ncut, GBL double *keep,
                                             VP *term, VP *mxs) {
    constexpr int U = WideTopo<CB>::U;
    constexpr uint32_t STEP = (uint32_t)U * kWave;
    const int last = d.T - 1;
    const uint32_t lo = uni(d.noff[last]), ln = uni(d.nn[last]);
    const int us = pool.ustride;
    const ParentVals<CB, PV_LDS> pv = parent_vals<CB, PV_LDS>(d, bv, last - 1);
    double tmx[CB], vmx[CB];
#pragma unroll
    for (int c = 0; c < CB; c++) { tmx[c] = -INFINITY; vmx[c] = -INFINITY; }
    auto load_topo = [&](uint32_t base, WideTopo<CB> &tp) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + (uint32_t)u * kWave + lane();
            const uint32_t ic = i < ln ? i : 0u;
            tp.t[u] = d.ntopo[lo + ic];
            tp.f[u] = i < ln ? (uint32_t)d.nflag[lo + ic] : 0u;
        }
    };
    // parent values and the previous terminal weights of one step
    auto load_px = [&](uint32_t base, const WideTopo<CB> &tp, double (&px)[U][CB], double (&w)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + (uint32_t)u * kWave + lane();
            const uint32_t ic = i < ln ? i : 0u;
            pv.load((tp.f[u] & kAlive) ? (tp.t[u] & kParentMask) : 0u, px[u]);
            w[u] = PASS_A ? d.tw[lo + ic] : keep[(size_t)ic * CB];
        }
    };
    WideTopo<CB> ta, tb;
    double pxa[U][CB], wa[U];
    load_topo(0, ta);
    load_px(0, ta, pxa, wa);
    load_topo(STEP, tb);
    for (uint32_t base = 0; base < ln; base += STEP) {
        double pxb[U][CB], wb[U];
        load_px(base + STEP, tb, pxb, wb);
        WideTopo<CB> tn;
        load_topo(base + 2 * STEP, tn);
        double cf[U][CB];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int c = 0; c < CB; c++) cf[u][c] = bv.coef[c * us + (ta.t[u] >> kRankShift)];
        sched_fence();
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + (uint32_t)u * kWave + lane();
            const bool alive = (ta.f[u] & kAlive) != 0;
            const uint32_t r = ta.t[u] >> kRankShift;
            const bool inal = (ta.f[u] & kInAlive) != 0;
            double ww = wa[u];
#pragma unroll
            for (int c = 0; c < CB; c++) {
                const double v = !inal ? DMIN : ((r != 0) ? pxa[u][c] + cf[u][c] : pxa[u][c]);
                const double nw = smin(ww, v);
                if (c < ncut) ww = nw;
                if (PASS_A) {
                    const bool use = alive & (c < ncut);
                    tmx[c] = (use && ww > tmx[c]) ? ww : tmx[c];
                    vmx[c] = (use && v > vmx[c]) ? v : vmx[c];
                }
            }
            if (alive) {
                if (PASS_A) keep[(size_t)i * CB] = wa[u];
                d.tw[lo + i] = ww;
            }
        }
        ta = tb;
        tb = tn;
#pragma unroll
        for (int u = 0; u < U; u++) {
            wa[u] = wb[u];
#pragma unroll
            for (int c = 0; c < CB; c++) pxa[u][c] = pxb[u][c];
        }
    }
    wave_mem_sync();
    if (PASS_A) {
#pragma unroll
        for (int c = 0; c < CB; c++) {
            tmx[c] = lane_reduce<1>(tmx[c], [](double a, double b) { return (b > a) ? b : a; });
            vmx[c] = lane_reduce<1>(vmx[c], [](double a, double b) { return (b > a) ? b : a; });
            term[c] = VP{tmx[c], tmx[c] != -INFINITY ? 0 : INT_MIN};
            mxs[c] = VP{vmx[c], vmx[c] != -INFINITY ? 0 : INT_MIN};
        }
#pragma unroll
        for (int c = 0; c < CB; c++)
            if (c < ncut && (tmx[c] == 0.0 || vmx[c] == 0.0))
                fused_leaf_pick<CB, PV_LDS>(d, bv, pool, ncut, keep, c, term[c], mxs[c]);
    }
}

template <int CB, bool PASS_A>
__device__ __forceinline__ void fused_leaf(const DD &d, BatchView &bv, const Pool &pool, int ncut, GBL double *keep,
                                           VP *term, VP *mxs) {
    if (d.T - 2 < d.kg) fused_leaf_t<CB, PASS_A, true>(d, bv, pool, ncut, keep, term, mxs);
    else fused_leaf_t<CB, PASS_A, false>(d, bv, pool, ncut, keep, term, mxs);
}

// Feasibility batch, last layer.  One streaming pass (as sweep_tail_layer_t) computes
// every alive leaf's values for the nb batch cuts and the first batch cut that removes it
// (state2 < -0.01, DD.cpp:3884-3889), stored as cut + 1 in nflag bits 3..7 (0: none);
// per cut it counts the removals and takes maxState over the leaves that survive the cut.
// Removing leaves never changes the values of the others, so the per-cut replay needs no
// further leaf values: dd_cascade(d, c + 1) removes cut c's leaves.  maxState is a plain
// maximum; for a zero maximum f_leaf_pick recomputes the reference's ordered pick.
template <int CB, bool PV_LDS>
__device__ __forceinline__ void f_leaf_pick(const DD &d, const BatchView &bv, const Pool &pool, int c, double &maxState) {
    const int last = d.T - 1;
    const uint32_t lo = uni(d.noff[last]), ln = uni(d.nn[last]);
    const int us = pool.ustride;
    const ParentVals<CB, PV_LDS> pv = parent_vals<CB, PV_LDS>(d, bv, last - 1);
    VP mx{0.0, INT_MIN};
    for (uint32_t i = lane(); i < ln; i += kWave) {
        const uint32_t f = d.nflag[lo + i];
        const uint32_t code = f >> 3;
        if (!(f & kAlive) || (code != 0 && code <= (uint32_t)c + 1u)) continue;
        const uint32_t t = d.ntopo[lo + i], r = t >> kRankShift;
        double px[CB];
        pv.load(t & kParentMask, px);
        const double v = !(f & kInAlive) ? DMIN : (r != 0 ? px[c] + bv.coef[c * us + r] : px[c]);
        mx = vp_pick(mx, VP{v, prio_old((int)i)});
    }
    mx = wave_vp(mx);
    maxState = (mx.p == INT_MIN) ? DMIN : smax(DMIN, mx.v);
}

template <int CB, bool PV_LDS>
__device__ __forceinline__ void f_leaf_scan_t(DD &d, BatchView &bv, const Pool &pool, int nb, int kS, uint32_t (&rm)[CB],
                                              double (&maxState)[CB]) {
    constexpr int U = WideTopo<CB>::U;
    constexpr uint32_t STEP = (uint32_t)U * kWave;
    const int last = d.T - 1;
    const uint32_t lo = uni(d.noff[last]), ln = uni(d.nn[last]);
    const int us = pool.ustride;
    const bool wr = kS >= d.T;   // state2 of the last batch cut, as sweep_tail_layer_t
    const ParentVals<CB, PV_LDS> pv = parent_vals<CB, PV_LDS>(d, bv, last - 1);
    uint32_t cnt[CB];
    double vmx[CB];
#pragma unroll
    for (int c = 0; c < CB; c++) { cnt[c] = 0; vmx[c] = -INFINITY; }
    auto load_topo = [&](uint32_t base, WideTopo<CB> &tp) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + (uint32_t)u * kWave + lane();
            const uint32_t ic = i < ln ? i : 0u;
            tp.t[u] = d.ntopo[lo + ic];
            tp.f[u] = i < ln ? (uint32_t)d.nflag[lo + ic] : 0u;
        }
    };
    auto load_px = [&](const WideTopo<CB> &tp, double (&px)[U][CB]) {
#pragma unroll
        for (int u = 0; u < U; u++) pv.load((tp.f[u] & kAlive) ? (tp.t[u] & kParentMask) : 0u, px[u]);
    };
    WideTopo<CB> ta, tb;
    double pxa[U][CB];
    load_topo(0, ta);
    load_px(ta, pxa);
    load_topo(STEP, tb);
    for (uint32_t base = 0; base < ln; base += STEP) {
        double pxb[U][CB];
        load_px(tb, pxb);
        WideTopo<CB> tn;
        load_topo(base + 2 * STEP, tn);
        double cf[U][CB];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int c = 0; c < CB; c++) cf[u][c] = bv.coef[c * us + (ta.t[u] >> kRankShift)];
        sched_fence();
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + (uint32_t)u * kWave + lane();
            const uint32_t f = ta.f[u];
            if (!(f & kAlive)) continue;
            const uint32_t r = ta.t[u] >> kRankShift;
            const bool inal = (f & kInAlive) != 0;
            double v[CB];
            int kc = nb;
#pragma unroll
            for (int c = CB - 1; c >= 0; c--) {
                v[c] = !inal ? DMIN : (r != 0 ? pxa[u][c] + cf[u][c] : pxa[u][c]);
                if (c < nb && v[c] < -0.01) kc = c;
            }
#pragma unroll
            for (int c = 0; c < CB; c++) {
                cnt[c] += (kc == c) ? 1u : 0u;
                vmx[c] = (kc > c && v[c] > vmx[c]) ? v[c] : vmx[c];
            }
            d.nflag[lo + i] = (uint8_t)((f & 7u) | (kc < nb ? (uint32_t)(kc + 1) << 3 : 0u));
            if (wr) {
                double w = v[0];
#pragma unroll
                for (int c = 1; c < CB; c++) w = (c == nb - 1) ? v[c] : w;
                d.s2[lo + i] = w;
            }
        }
        ta = tb;
        tb = tn;
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int c = 0; c < CB; c++) pxa[u][c] = pxb[u][c];
    }
#pragma unroll
    for (int c = 0; c < CB; c++) {
        rm[c] = wave_sum(cnt[c]);
        vmx[c] = lane_reduce<1>(vmx[c], [](double a, double b) { return (b > a) ? b : a; });
        maxState[c] = (vmx[c] == -INFINITY) ? DMIN : smax(DMIN, vmx[c]);
    }
    wave_mem_sync();
#pragma unroll
    for (int c = 0; c < CB; c++)
        if (c < nb && vmx[c] == 0.0) f_leaf_pick<CB, PV_LDS>(d, bv, pool, c, maxState[c]);
}

template <int CB>
__device__ __forceinline__ void f_leaf_scan(DD &d, BatchView &bv, const Pool &pool, int nb, int kS, uint32_t (&rm)[CB],
                                            double (&maxState)[CB]) {
    if (d.T - 2 < d.kg) f_leaf_scan_t<CB, true>(d, bv, pool, nb, kS, rm, maxState);
    else f_leaf_scan_t<CB, false>(d, bv, pool, nb, kS, rm, maxState);
}

// getPathForNode (DD.cpp:3796-3820): walk up, first in-arc whose parent.state2 + weight
// equals this node's state2; if none matches, continue through the first in-arc
// without recording a decision.  Decisions land in d.walk (bottom-up); returns count.
__device__ __forceinline__ int dd_walk(const NetDev &net, DD &d, uint32_t node, int k, const GBL double *row) {
    int cnt = 0;
    while (k > 0) {
        const uint32_t pnoff = uni(d.noff[k - 1]);
        const uint32_t acnt = uni(d.acnt[k]);
        const double cur = acnt ? d.s2[node] : 0.0;
        uint32_t parent;
        int found = 0;
        int16_t dec = 0;
        if (acnt) {
            const uint32_t aoff = uni(d.aoff[k]);
            uint32_t first_alive = 0xFFFFFFFFu, match = 0xFFFFFFFFu;
            for (uint32_t base = 0; base < acnt && match == 0xFFFFFFFFu; base += kWave) {
                uint32_t a = base + lane();
                bool alive = a < acnt && (d.aflag[aoff + a] & kAlive);
                bool hit = false;
                if (alive) {
                    uint32_t t = d.atopo[aoff + a];
                    uint32_t p = t & kParentMask, r = t >> kRankShift;
                    hit = (d.s2[pnoff + p] + arc_weight(net, d, k, (int)r, row)) == cur;
                }
                uint64_t ba = __ballot(alive), bh = __ballot(hit);
                if (first_alive == 0xFFFFFFFFu && ba) first_alive = base + (uint32_t)(__ffsll((unsigned long long)ba) - 1);
                if (bh) match = base + (uint32_t)(__ffsll((unsigned long long)bh) - 1);
            }
            uint32_t pick = (match != 0xFFFFFFFFu) ? match : first_alive;
            if (pick == 0xFFFFFFFFu) break;  // no incoming arc left (reference: UB)
            uint32_t t = d.atopo[uni(d.aoff[k]) + pick];
            parent = pnoff + (t & kParentMask);
            if (match != 0xFFFFFFFFu) {
                found = 1;
                dec = rank_value(net, d.g + k - 1, (int)(t >> kRankShift));
            }
        } else {
            // A single incoming arc: its parent.state2 + weight is exactly how this node's
            // state2 was computed in the same sweep, so the reference's equality test
            // (DD.cpp:3808) always holds for it; no state2 is read here.
            uint32_t t = d.ntopo[node];
            uint32_t p = t & kParentMask, r = t >> kRankShift;
            parent = pnoff + p;
            if (d.nflag[node] & kInAlive) {
                found = 1;
                dec = rank_value(net, d.g + k - 1, (int)r);
            }
        }
        if (found) {
            if (lane() == 0) d.walk[cnt] = dec;
            cnt++;
        }
        node = parent;
        k--;
    }
    wave_lds_sync();
    return cnt;
}

__device__ __forceinline__ void load_meta_layers(DD &d, const Scratch &sc, int slot) {
    const GBL int32_t *meta = sc.meta + (size_t)slot * 8;
    d.g = uni(meta[0]); d.len = uni(meta[1]); d.T = uni(meta[2]); d.exact = uni(meta[3]); d.aligned = uni(meta[4]);
    const GBL uint32_t *lay = sc.lay + (size_t)slot * sc.Tcap * 5;
    for (int k = lane(); k < d.T; k += kWave) {
        d.noff[k] = lay[k]; d.nn[k] = lay[sc.Tcap + k]; d.nalive[k] = lay[2 * sc.Tcap + k];
        d.aoff[k] = lay[3 * sc.Tcap + k]; d.acnt[k] = lay[4 * sc.Tcap + k];
    }
    wave_mem_sync();
}

__device__ __forceinline__ void store_meta_layers(const DD &d, const Scratch &sc, int slot, int last_cut, int status,
                                         int cut_layer, double ub) {
    GBL int32_t *meta = sc.meta + (size_t)slot * 8;
    if (lane() == 0) {
        meta[0] = d.g; meta[1] = d.len; meta[2] = d.T; meta[3] = d.exact; meta[4] = d.aligned;
        meta[5] = last_cut; meta[6] = status; meta[7] = cut_layer;
        sc.ubv[slot] = ub;
    }
    GBL uint32_t *lay = sc.lay + (size_t)slot * sc.Tcap * 5;
    for (int k = lane(); k < d.T; k += kWave) {
        lay[k] = (d.noff[k]); lay[sc.Tcap + k] = (d.nn[k]); lay[2 * sc.Tcap + k] = (d.nalive[k]);
        lay[3 * sc.Tcap + k] = (d.aoff[k]); lay[4 * sc.Tcap + k] = (d.acnt[k]);
    }
}

// exact DD: argmax terminal arc (strict >, first wins) then the path of its tail
__device__ __forceinline__ int dd_solution_path(const NetDev &net, DD &d, const GBL double *row, GBL int16_t *out_path,
                                const GBL int16_t *rsol) {
    const int last = d.T - 1;
    const uint32_t lo = uni(d.noff[last]), ln = uni(d.nn[last]);
    VP best{0.0, INT_MIN};
    for (uint32_t base = 0; base < ln; base += kWave) {
        uint32_t i = base + lane();
        if (i < ln && (d.nflag[lo + i] & kAlive)) best = vp_pick(best, VP{d.tw[lo + i], prio_old((int)i)});
    }
    best = wave_vp(best);
    uint32_t node = 0;
    int k = 0;
    if (best.p != INT_MIN && best.v > DMIN) {
        node = lo + (uint32_t)(-best.p - 2);
        k = last;
    }
    int cnt = dd_walk(net, d, node, k, row);
    for (int t = lane(); t < d.len; t += kWave) out_path[t] = rsol[t];
    for (int t = lane(); t < cnt; t += kWave) out_path[d.len + t] = d.walk[cnt - 1 - t];
    return d.len + cnt;
}

// ------------------------------------------------------------------------------------
// Pool order: the feasibility list then the optimality list, each newest first
// (NodeExplorer.cpp:935-944 / 975-983).
__device__ __forceinline__ int seq_id(const Pool &pool, int s) { return s < pool.nf ? pool.f_order[s] : pool.o_order[s - pool.nf]; }

// Root prefix (DD.cpp:3938-3949): v = RHS, then v = v + coef for each decision of the
// record's solution vector in order, skipping -1.  The fold is sequential; its loads are
// independent, so they are issued kFoldBatch at a time ahead of the adds.
constexpr int kFoldBatch = 16;
__device__ __forceinline__ double root_fold(const GBL double *row, double v, const DD &d) {
    for (int t0 = 0; t0 < d.len; t0 += kFoldBatch) {
        double x[kFoldBatch];
        bool ok[kFoldBatch];
#pragma unroll
        for (int j = 0; j < kFoldBatch; j++) {
            const int t = t0 + j;
            const int sl = t < d.len ? (int)d.rslot[t] : -1;
            ok[j] = sl >= 0;
            x[j] = row[ok[j] ? sl : 0];
        }
        sched_fence();
#pragma unroll
        for (int j = 0; j < kFoldBatch; j++)
            if (ok[j]) v = v + x[j];
    }
    return v;
}

// root fold of the cuts at pool positions s0 + lane (lanes past the pool fold the last)
__device__ __forceinline__ double root_fold_seq(const Pool &pool, const DD &d, int s0, int total) {
    const int s = min(s0 + lane(), total - 1);
    const int id = seq_id(pool, s);
    return root_fold(pool.rows + (size_t)id * pool.stride, pool.rhs[id], d);
}

struct LoopState {
    int status;
    double ub;
    int last_cut;
    uint32_t applied;
    uint32_t redo;
#ifdef SGUFP_PHASES
    uint64_t ph[8];   // diagnostic ticks per phase (see BatchOut::phase)
    uint64_t t;       // last stamp
    __device__ __forceinline__ void stamp(int k) {
        uint64_t now = wall_clock64();
        ph[k] += now - t;
        t = now;
    }
#else
    // the production build keeps no clock stamps in the hot kernel (lib_prof/ has them)
    __device__ __forceinline__ void stamp(int) {}
#endif
};

// ------------------------------------------------------------------------------------
// Hand-off of a non-exact DD to the cut-parallel optimality phase (kNxPending, see
// dd_device.hpp).  k_nx_dag sweeps the layers 1 .. k0 (k0 = the last width-1 layer <= T-2)
// layer by layer with lanes = (node group, cut) from the packed topology words build_stream
// left in the slot (tmir: every layer below kg has <= 127 nodes); the leaf passes take the
// tree below k0.  Kept back (the record stays in k_relax): k0 at or past kg, more than
// kNxRanks + 1 state ranks, or a deeper / wider tail than the leaf passes stage.
// diagnostics: ExactIO::ctr[9] counts the DDs kept back, 10 bits per reason
__device__ __forceinline__ bool nx_refuse(const ExactIO &ex, int why) {
    if (lane() == 0) atomicAdd(&ex.ctr[9], 1ull << (10 * why));
    return false;
}

__device__ bool nx_compile(const DD &d, const Scratch &sc, const ExactIO &ex, int slot, int &k0_out, int first) {
    const int T = d.T;
    if (T < 3 || d.us > kNxRanks + 1 || !d.stream) return nx_refuse(ex, 0);
    int k0 = 0;
    for (int base = 0; base <= T - 2; base += kWave) {
        const int k = base + lane();
        const uint64_t b = __ballot(k <= T - 2 && d.nalive[k] == 1u);
        if (b) k0 = base + 63 - __clzll((long long)b);
    }
    k0 = uni(k0);
    const int D = T - 1 - k0;
    if (D < 1 || D > kExactMaxT - 1 || D * d.us > kExactMaxEntries) return nx_refuse(ex, 1);
    if (k0 >= d.kg) return nx_refuse(ex, 2);
    // the single alive node of layer k0 (its index: the leaf passes' root)
    const uint32_t noff = uni(d.noff[k0]), n = uni(d.nn[k0]);
    uint32_t q = 0xFFFFFFFFu;
    for (uint32_t base = 0; base < n && q == 0xFFFFFFFFu; base += kWave) {
        const uint32_t i = base + lane();
        const uint64_t b = __ballot(i < n && (d.nflag[noff + i] & kAlive));
        if (b) q = base + (uint32_t)(__ffsll((unsigned long long)b) - 1);
    }
    if (q == 0xFFFFFFFFu) return nx_refuse(ex, 3);
    if (lane() == 0) {
        GBL int32_t *h = ex.nxh + (size_t)slot * 4;
        h[0] = k0;
        h[1] = (int32_t)d.Nn;
        h[2] = (int32_t)q;
        h[3] = first;   // the first pool position (O list, newest first) the phase applies
    }
    k0_out = k0;
    return true;
}

// one cut at a time from pool position s onwards; efast: an exact DD leaves at the first
// optimality cut for the cut-parallel kernels (kExactPending, exact_kernels.hip)
__device__ __forceinline__ void cut_loop_single(const NetDev &net, DD &d, const Pool &pool, double incumbent, int s, LoopState &st,
                                                bool efast = false) {
    const int total = pool.nf + pool.no;
    if (efast && s >= pool.nf) { st.status = kExactPending; return; }
    for (int s0 = s; s0 < total; s0 += kWave) {
        double rv = root_fold_seq(pool, d, s0, total);
        int cnt = min(kWave, total - s0);
        for (int j = 0; j < cnt; j++) {
            const int seq = s0 + j;
            if (efast && seq >= pool.nf) { st.status = kExactPending; return; }
            const int id = seq_id(pool, seq);
            const GBL double *row = pool.rows + (size_t)id * pool.stride;
            dd_sweep(net, d, row, lane_get(rv, j));
            st.stamp(1);
            st.last_cut = id;
            st.applied++;
            if (seq < pool.nf) {
                if (!dd_post_feasibility(net, d, row)) { st.status = kPrunedFeasibility; return; }
            } else {
                double v = dd_post_optimality(net, d, row, incumbent);
                st.ub = d.exact ? v : smin(v, st.ub);
                if (st.ub <= incumbent) { st.status = kPrunedOptimality; return; }
            }
            st.stamp(4);
        }
    }
}

// Width-1 pruning of cut `id` over the layers of the fire mask fm (DD.cpp:3895-3928 /
// 3987-4021): in each, every alive in-arc with parent.state2 + weight + gain <= thresh
// goes, gain = maxState - state2 of the layer's single node.  Marks use the sweep's
// state2 only and removing an arc of one layer changes nothing another layer reads, so
// the layers are processed back to back with their loads batched and no hand-off in
// between (removing them at once, as the reference's batchRemoveArcs, is the same).
// Returns false when some layer would lose all of its incoming arcs.
template <int CB>
__device__ __forceinline__ bool prune_layers(const NetDev &net, DD &d, const BatchView &bv, const Pool &pool, int id, int first,
                                             int end, double maxState, double thresh) {
    constexpr int U = 4;
    const int us = pool.ustride;
    const GBL double *ct = pool.coefT + (size_t)id * ((size_t)net.L * us);
    bool ok = true;
    for (int wb = first & ~63; wb < end && ok; wb += kWave) {
        uint64_t b = bv.fm[wb >> 6];
        while (b && ok) {
            const int k = wb + (int)(__ffsll((unsigned long long)b) - 1);
            b &= b - 1;
            const uint32_t pnoff = uni(d.noff[k - 1]), acnt = uni(d.acnt[k]);
            const GBL double *ck = ct + (size_t)(d.g + k - 1) * us;
            uint32_t total = 0, pruned = 0;
            if (acnt) {
                const uint32_t aoff = uni(d.aoff[k]);
                const double gain = maxState - d.s2[uni(d.noff[k])];
                for (uint32_t base = 0; base < acnt; base += U * kWave) {
                    uint32_t fl[U], tp[U];
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const uint32_t a = base + (uint32_t)u * kWave + lane();
                        const uint32_t ac = a < acnt ? a : 0u;
                        fl[u] = a < acnt ? (uint32_t)d.aflag[aoff + ac] : 0u;
                        tp[u] = d.atopo[aoff + ac];
                    }
                    sched_fence();
                    double px[U], w[U];
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const uint32_t r = tp[u] >> kRankShift;
                        px[u] = d.s2[pnoff + (tp[u] & kParentMask)];
                        w[u] = r == 0 ? 0.0 : ck[r];
                    }
                    sched_fence();
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const uint32_t a = base + (uint32_t)u * kWave + lane();
                        const bool alive = (fl[u] & kAlive) != 0;
                        const bool pr = alive && ((px[u] + w[u]) + gain) <= thresh;
                        if (pr) {
                            d.aflag[aoff + a] = 0;
                            mir_arc_kill(d, aoff + a, tp[u] >> kRankShift);
                            __hip_atomic_fetch_sub(&d.outcnt[pnoff + (tp[u] & kParentMask)], 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                        }
                        total += (uint32_t)__popcll(__ballot(alive));
                        pruned += (uint32_t)__popcll(__ballot(pr));
                    }
                }
            } else {
                const uint32_t M = layer_single(d, k);
                const uint32_t t = d.ntopo[M], f = d.nflag[M];
                const uint32_t p = t & kParentMask, r = t >> kRankShift;
                const double sM = d.s2[M], px = d.s2[pnoff + p], w = r == 0 ? 0.0 : ck[r];
                if (f & kInAlive) {
                    total = 1;
                    if (((px + w) + (maxState - sM)) <= thresh) {
                        pruned = 1;
                        if (lane() == 0) {
                            d.nflag[M] = (uint8_t)(f & ~kInAlive);
                            mir_node_clear(d, M, kMirIn);
                            d.outcnt[pnoff + p] -= 1u;
                        }
                    }
                }
            }
            if (total == pruned) ok = false;
        }
    }
    wave_mem_sync();
    return ok;
}

// Fire mask of the batch cut c over [first, end) from the summaries sm/xm (stride CB) into
// bv.fm; returns whether any layer fires.
template <int CB>
__device__ __forceinline__ bool fire_layers(const DD &d, BatchView &bv, int c, int first, int end, double thresh,
                                            double maxState) {
    const int nw = (d.T + 63) / 64;
    for (int w = lane(); w < nw; w += kWave) bv.fm[w] = 0;
    wave_lds_sync();
    uint64_t any = 0;
    for (int base = first; base < end; base += kWave) {
        const uint64_t b = prune_fire(d, base, end, maxState, thresh, bv.sm + c, bv.xm + c, CB, bv.w1);
        any |= b;
        if (b && lane() == 0) {
            // window [base, base + 64) may straddle two words
            const int w0 = base >> 6, sh = base & 63;
            bv.fm[w0] |= b << sh;
            if (sh && w0 + 1 < nw) bv.fm[w0 + 1] |= b >> (64 - sh);
        }
    }
    wave_lds_sync();
    return any != 0;
}

// Exact redo of one cut whose width-1 pruning fires (batch cut c, pool row id): a sweep
// with this cut alone, then the pruning (DD.cpp:3895-3928 / 3987-4021).  The pruning reads
// state2 only in the firing layers and the layers above them; those are known before the
// sweep from the batch summaries of cut c (same DD, same values), so the sweep writes
// state2 of just those layers; the summaries the sweep recomputes must fire the same
// layers (checked; otherwise the sweep is repeated writing every layer).  Returns false
// when a width-1 layer would lose all of its incoming arcs.
template <int CB>
__device__ __forceinline__ bool redo_cut(const NetDev &net, DD &d, BatchView &bv, const Pool &pool, int c, int id,
                                         double rv1, int first, int end, double thresh, double maxState,
                                         bool unchanged) {
    const int last = d.T - 1;
    const int nw = (d.T + 63) / 64;
    fire_layers<CB>(d, bv, c, first, end, thresh, maxState);
    for (int w = lane(); w < nw; w += kWave) {
        const uint64_t f = bv.fm[w], fn = w + 1 < nw ? bv.fm[w + 1] : 0ull;
        bv.wm[w] = f | (f >> 1) | (fn << 63);   // layer k fires -> write k and k - 1
    }
    if (lane() == 0) bv.ids[0] = id;
    for (int k = lane(); k < d.T; k += kWave) bv.w1[k] = ((d.nalive[k]) == 1) ? 1 : 0;
    wave_lds_sync();
    if (unchanged) {
        // no edit since the batch sweep: the fresh summaries equal the batch ones, so the
        // fire mask stands and the sweep stops after the last layer it writes
        int kend = 0;
        for (int w = 0; w < nw; w++) {
            const uint64_t m = bv.wm[w];
            if (m) kend = w * 64 + 64 - (int)__clzll((long long)m);
        }
        bv.wsel = bv.wm;
        sweep_narrow<CB>(net, d, bv, pool, 1, rv1, d.T, kend);
        if (d.kg == 0 && lane() == 0) bv.s2b[0] = rv1;
        for (int k = max(d.kg, 1); k < min(last, kend); k++) sweep_tail_layer<CB>(net, d, bv, pool, k, 1, d.T);
        bv.wsel = nullptr;
        wave_mem_sync();
        return prune_layers<CB>(net, d, bv, pool, id, first, end, maxState, thresh);
    }
    for (int attempt = 0; attempt < 2; attempt++) {
        bv.wsel = bv.wm;
        sweep_narrow<CB>(net, d, bv, pool, 1, rv1, d.T);
        if (d.kg == 0 && lane() == 0) bv.s2b[0] = rv1;
        for (int k = max(d.kg, 1); k < last; k++) sweep_tail_layer<CB>(net, d, bv, pool, k, 1, d.T);
        bv.wsel = nullptr;
        wave_mem_sync();
        // the fire mask of the fresh summaries must lie inside the write mask
        bool covered = true;
        fire_layers<CB>(d, bv, 0, first, end, thresh, maxState);
        for (int w = 0; w < nw; w++) {
            const uint64_t f = bv.fm[w], fn = w + 1 < nw ? bv.fm[w + 1] : 0ull;
            if (((f | (f >> 1) | (fn << 63)) & ~bv.wm[w]) != 0) covered = false;
        }
        if (covered) break;
        for (int w = lane(); w < nw; w += kWave) bv.wm[w] = ~0ull;
        wave_lds_sync();
    }
    return prune_layers<CB>(net, d, bv, pool, id, first, end, maxState, thresh);
}

// CB cuts of one type per sweep, replayed in pool order (see "Multi-cut sweeps")
// ------------------------------------------------------------------------------------
// Optimality-cut screening.  After the feasibility phase the reference applies the O cuts
// newest first and prunes as soon as ub <= optimalLB, where after cut j
//     ub <= terminalState_j = max_leaf min_{i <= j} state2'_i(leaf)
// (running minimum on every terminal arc, DD.cpp:3975-3984) and state2' is computed on
// the DD the earlier O cuts edited.  Those edits only remove arcs, and rounding is
// monotone, so state2'_i(leaf) <= v_i(leaf), the longest-path value of cut i on the
// post-feasibility DD without any O edit.  Hence, for any set S of O cuts,
//     max_leaf min_{i in S} v_i(leaf) <= optimalLB   ==>   the reference prunes the node
// (status PRUNED_BY_OPTIMALITY_CUT, lb = ub = DOUBLE_MIN) at or before the last cut of S.
// The screen sweeps the few strongest cuts first (o_rank: ascending node-independent
// upper bound RHS + sum_l max_r coef) with a per-leaf running minimum; when it proves
// the prune the exact optimality phase is skipped, otherwise the exact phase runs as if
// nothing happened (the screen writes no DD state the exact phase reads).

// leaf values of the nb screening cuts: run[i] = min(run[i], v_c(i)); returns the max over
// alive leaves of run (DMIN when none is alive).  Streaming as in sweep_tail_layer_t.
template <int CB, bool PV_LDS>
__device__ __forceinline__ double screen_leaf_t(const DD &d, BatchView &bv, const Pool &pool, int nb, bool first,
                                                GBL double *run) {
    constexpr int U = WideTopo<CB>::U;
    constexpr uint32_t STEP = (uint32_t)U * kWave;
    const int last = d.T - 1;
    const uint32_t lo = uni(d.noff[last]), ln = uni(d.nn[last]);
    const int us = pool.ustride;
    const ParentVals<CB, PV_LDS> pv = parent_vals<CB, PV_LDS>(d, bv, last - 1);
    double best = -INFINITY;
    auto load_topo = [&](uint32_t base, WideTopo<CB> &tp) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + (uint32_t)u * kWave + lane();
            const uint32_t ic = i < ln ? i : 0u;
            tp.t[u] = d.ntopo[lo + ic];
            tp.f[u] = i < ln ? (uint32_t)d.nflag[lo + ic] : 0u;
        }
    };
    auto load_px = [&](uint32_t base, const WideTopo<CB> &tp, double (&px)[U][CB], double (&m)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + (uint32_t)u * kWave + lane();
            const uint32_t ic = i < ln ? i : 0u;
            pv.load((tp.f[u] & kAlive) ? (tp.t[u] & kParentMask) : 0u, px[u]);
            m[u] = first ? DMAX : run[(size_t)ic * CB];
        }
    };
    WideTopo<CB> ta, tb;
    double pxa[U][CB], ma[U];
    load_topo(0, ta);
    load_px(0, ta, pxa, ma);
    load_topo(STEP, tb);
    for (uint32_t base = 0; base < ln; base += STEP) {
        double pxb[U][CB], mb[U];
        load_px(base + STEP, tb, pxb, mb);
        WideTopo<CB> tn;
        load_topo(base + 2 * STEP, tn);
        double cf[U][CB];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int c = 0; c < CB; c++) cf[u][c] = bv.coef[c * us + (ta.t[u] >> kRankShift)];
        sched_fence();
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t i = base + (uint32_t)u * kWave + lane();
            const bool alive = (ta.f[u] & kAlive) != 0, inal = (ta.f[u] & kInAlive) != 0;
            const uint32_t r = ta.t[u] >> kRankShift;
            double m = ma[u];
#pragma unroll
            for (int c = 0; c < CB; c++) {
                if (c < nb) {
                    const double v = !inal ? DMIN : ((r != 0) ? pxa[u][c] + cf[u][c] : pxa[u][c]);
                    m = fmin(m, v);
                }
            }
            if (alive) {
                run[(size_t)i * CB] = m;
                best = (m > best) ? m : best;
            }
        }
        ta = tb;
        tb = tn;
#pragma unroll
        for (int u = 0; u < U; u++) {
            ma[u] = mb[u];
#pragma unroll
            for (int c = 0; c < CB; c++) pxa[u][c] = pxb[u][c];
        }
    }
    best = lane_reduce<1>(best, [](double a, double b) { return (b > a) ? b : a; });
    wave_mem_sync();
    return best != -INFINITY ? best : DMIN;
}

template <int CB>
__device__ __forceinline__ double screen_leaf(const DD &d, BatchView &bv, const Pool &pool, int nb, bool first,
                                              GBL double *run) {
    if (d.T - 2 < d.kg) return screen_leaf_t<CB, true>(d, bv, pool, nb, first, run);
    return screen_leaf_t<CB, false>(d, bv, pool, nb, first, run);
}

// root fold (DD.cpp:3938-3949) of pool row `id` (lane-uniform or per lane)
__device__ __forceinline__ double root_fold_row(const Pool &pool, const DD &d, int id) {
    return root_fold(pool.rows + (size_t)id * pool.stride, pool.rhs[id], d);
}

// true: the screen proves the optimality prune
template <int CB>
__device__ __forceinline__ bool screen_opt(const NetDev &net, DD &d, BatchView &bv, const Pool &pool, double incumbent,
                                           LoopState &st) {
    const int last = d.T - 1;
    GBL double *run = bv.s2b + (size_t)(uni(d.noff[last]) - bv.gbase) * CB;   // last-layer region, free here
    const int n = min(pool.nscreen, pool.no);
    for (int sp = 0; sp < n; sp += CB) {
        const int nb = min(CB, n - sp);
        if (lane() < nb) bv.ids[lane()] = pool.o_rank[sp + lane()];
        for (int k = lane(); k < d.T; k += kWave) bv.w1[k] = ((d.nalive[k]) == 1) ? 1 : 0;
        const double rv = root_fold_row(pool, d, pool.o_rank[sp + min(lane(), nb - 1)]);
        wave_lds_sync();
        sweep_narrow<CB>(net, d, bv, pool, nb, rv, 0);
        if (d.kg == 0 && lane() < nb) bv.s2b[lane()] = rv;
        for (int k = max(d.kg, 1); k < last; k++) sweep_tail_layer<CB>(net, d, bv, pool, k, nb, 0);
        batch_coef_direct(net, d, bv, pool, last, nb);
        const double u = screen_leaf<CB>(d, bv, pool, nb, sp == 0, run);
        st.applied += (uint32_t)nb;
        if (u <= incumbent) return true;
    }
    return false;
}

template <int CB>
__device__ __forceinline__ void cut_loop_batched(const NetDev &net, DD &d, const Scratch &sc, BatchView &bv, const Pool &pool,
                                 double incumbent, LoopState &st, bool efast, const ExactIO *nx = nullptr, int slot = 0,
                                 int *nx_k0 = nullptr) {
    const int total = pool.nf + pool.no;
    const int last = d.T - 1;
    bv.gbase = uni(d.noff[d.kg]);
    if (d.T < 2 || uni(d.noff[last]) + uni(d.nn[last]) - bv.gbase > (uint32_t)sc.tail_cap) {
        cut_loop_single(net, d, pool, incumbent, 0, st, efast);
        return;
    }
    int s = 0;
    bool screened = pool.nscreen <= 0;
    while (s < total) {
        const bool feas = s < pool.nf;
        if (!feas && !screened) {
            screened = true;
            const bool pruned = screen_opt<CB>(net, d, bv, pool, incumbent, st);
            st.stamp(6);
            if (pruned) { st.status = kPrunedOptimality; return; }
        }
        if (!feas && efast) { st.status = kExactPending; return; }
        // a non-exact DD under a large pool that survived the first nx_skip optimality cuts in
        // order (most records that a cut prunes go there, cheaply): the cut-parallel phase takes
        // the rest of the pool from here (once)
        if (!feas && nx && s >= pool.nf + nx->nx_skip) {
            if (nx_compile(d, sc, *nx, slot, *nx_k0, s - pool.nf)) { st.status = kNxPending; return; }
            nx = nullptr;
        }
        const int nb = min(CB, (feas ? pool.nf : total) - s);
        if (lane() < nb) bv.ids[lane()] = seq_id(pool, s + lane());
        for (int k = lane(); k < d.T; k += kWave) bv.w1[k] = ((d.nalive[k]) == 1) ? 1 : 0;
        int kS = d.T;
        for (int base = 3; base < d.T; base += kWave) {
            int k = base + lane();
            uint64_t b = __ballot(k < d.T && (d.nalive[k]) == 1);
            if (b) { kS = base + (int)(__ffsll((unsigned long long)b) - 1) + 1; break; }
        }
        const double rv = root_fold_seq(pool, d, s, total);
        wave_lds_sync();
        st.stamp(4);
        sweep_narrow<CB>(net, d, bv, pool, nb, rv, kS);
        st.stamp(1);
        if (d.kg == 0 && lane() < nb) bv.s2b[lane()] = rv;
        for (int k = max(d.kg, 1); k < last; k++) sweep_tail_layer<CB>(net, d, bv, pool, k, nb, kS);
        st.stamp(2);
        int next = s + nb;
        if (feas) {
            // feasibility cuts: one scan of the last layer (first removing cut per leaf),
            // then removal + cascade replayed per cut
            batch_coef_direct(net, d, bv, pool, last, nb);
            uint32_t rm[CB];
            double mstate[CB];
            f_leaf_scan<CB>(d, bv, pool, nb, kS, rm, mstate);
            st.stamp(3);
            bool removed = false;   // some batch cut so far removed leaves (the DD changed)
            for (int c = 0; c < nb; c++) {
                const int seq = s + c;
                const int id = uni(bv.ids[c]);
                st.last_cut = id;
                st.applied++;
                double maxState = DMIN;
#pragma unroll
                for (int cc = 0; cc < CB; cc++) maxState = (cc == c) ? mstate[cc] : maxState;
                uint32_t rmc = 0;
#pragma unroll
                for (int cc = 0; cc < CB; cc++) rmc = (cc == c) ? rm[cc] : rmc;
                if (rmc == uni(d.nalive[last])) { st.status = kPrunedFeasibility; return; }
                if (rmc) { dd_cascade(d, (uint32_t)c + 1u); removed = true; }
                if (!d.exact && dd_prune_check<CB>(d, bv, c, 1, last, -0.01, maxState)) {
                    st.stamp(4);
                    if (!redo_cut<CB>(net, d, bv, pool, c, id, lane_get(rv, c), 1, last, -0.01, maxState, !removed)) {
                        st.status = kPrunedFeasibility;
                        return;
                    }
                    st.stamp(5);
                    next = seq + 1;
                    st.redo++;
                    break;
                }
            }
            st.stamp(4);
        } else {
            // optimality cuts: fused last layer (pass A: terminal states, pass B: commit)
            batch_coef_direct(net, d, bv, pool, last, nb);
            VP term[CB], mxs[CB];
            GBL double *keep = bv.s2b + (size_t)(uni(d.noff[last]) - bv.gbase) * CB;  // free in O batches
            fused_leaf<CB, true>(d, bv, pool, nb, keep, term, mxs);
            st.stamp(3);
            // replay in pool order (unrolled: term / mxs stay in registers); the width-1
            // pruning tests of all batch cuts in one pass (no edit happens before a redo)
            int capply = nb - 1, redo = -1;
            bool stop = false, pruned = false;
            double redo_v = DMIN, redo_ms = DMIN;
            double mstate[CB];
#pragma unroll
            for (int c = 0; c < CB; c++) mstate[c] = (mxs[c].p == INT_MIN) ? DMIN : smax(DMIN, mxs[c].v);
            const uint32_t fire = d.exact ? 0u : dd_prune_mask<CB>(d, bv, 0, nb, 3, last - 1, incumbent - 0.01, mstate);
#pragma unroll
            for (int c = 0; c < CB; c++) {
                if (stop || c >= nb) continue;
                double v = (term[c].p == INT_MIN) ? DMIN : smax(DMIN, term[c].v);
                double maxState = mstate[c];
                if (v > incumbent && !d.exact && ((fire >> c) & 1u)) {
                    capply = c;
                    redo = c;
                    redo_v = v;
                    redo_ms = maxState;
                    stop = true;
                    continue;
                }
                st.applied++;
                st.last_cut = bv.ids[c];
                st.ub = d.exact ? v : smin(v, st.ub);
                if (st.ub <= incumbent) { stop = true; pruned = true; }
            }
            if (pruned) { st.status = kPrunedOptimality; return; }
            st.stamp(4);
            if (capply < nb - 1) {
                fused_leaf<CB, false>(d, bv, pool, capply + 1, keep, nullptr, nullptr);
                st.stamp(3);
            }
            if (redo >= 0) {
                const int c = redo;
                const int id = uni(bv.ids[c]);
                double v = redo_v;
                if (!redo_cut<CB>(net, d, bv, pool, c, id, lane_get(rv, c), 3, last - 1, incumbent - 0.01, redo_ms, true))
                    v = DMIN;
                st.applied++;
                st.last_cut = id;
                st.ub = d.exact ? v : smin(v, st.ub);
                if (st.ub <= incumbent) { st.status = kPrunedOptimality; return; }
                next = s + c + 1;
                st.redo++;
                st.stamp(5);
            }
        }
        s = next;
    }
}

// ------------------------------------------------------------------------------------
// Kernel 1: build + pool sweeps + finish, one wave per open node.
template <int CB>
__global__ void __launch_bounds__(kWave, 2) k_relax(NetDev net, Scratch sc, BatchIn in, Pool pool, BatchOut out,
                                                double incumbent, ExactIO ex) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS uint8_t *smem = (LDS uint8_t *)smem_raw;
    if ((int)blockIdx.x >= in.n) return;
    const int slot = in.perm ? in.perm[blockIdx.x] : (int)blockIdx.x;
    // the re-run after the cut-parallel phase of non-exact DDs: only the records it could
    // not settle (kNxFallback), in order, from scratch
    if (ex.redo && out.status[slot] != kNxFallback) return;
#ifdef SGUFP_PHASES
    const uint64_t t_start = wall_clock64();
#endif
    DD d;
    dd_bind(d, smem, sc, slot, CB);
    d.stream = 0;
    d.ng = 0;
    d.kg = 0;
    d.Nn = 0;
    d.Amir = 0;
    d.g = uni((int)in.gl[slot]);
    d.len = uni((int)in.sol_len[slot]);
    const GBL int16_t *rsol = in.sol + in.sol_off[slot];
    d.aligned = (d.len == d.g) ? 1 : 0;
    int cut_layer = 0;
#ifdef SGUFP_PHASES
    LoopState st{kSuccess, in.ub[slot], -1, 0, 0, {0, 0, 0, 0, 0, 0, 0, 0}, t_start};
#else
    LoopState st{kSuccess, in.ub[slot], -1, 0, 0};
#endif
    double lb = DMIN;
    uint32_t nchild = 0, n_nodes = 0, n_arcs = 0, n_merged = 0;
    bool efast = false;
    int nx_k0 = -1;
    d.T = 1; d.exact = 1;

    if (!in.valid[slot] || d.len > d.g || d.g > net.L || d.len > sc.Lcap) {
        st.status = kErrRecord;
        goto done;
    }
    if (in.bound_prune && in.ub[slot] <= incumbent) {   // DDSolver.cpp:707-711
        st.status = kPrunedBound;
        goto done;
    }
    // coefficient slots of the root solution (layer t, decision sol[t])
    for (int t = lane(); t < d.len; t += kWave) {
        int dec = rsol[t];
        int s = -1;
        if (dec != -1) {
            s = net.n_slots;
            if (dec >= 0 && dec < net.m) {
                int j = net.arc_head[dec];
                for (int q = net.slot_off[t]; q < net.slot_off[t + 1]; q++)
                    if (net.slot_head[q] == j) { s = q; break; }
            }
        }
        d.rslot[t] = (int16_t)s;
    }
    if (!dd_build(net, d, sc, in.mask[slot], n_nodes, n_arcs, n_merged)) {
        st.status = kErrCapacity;
        goto done;
    }
    st.stamp(0);
    // exact DDs whose optimality phase the cut-parallel kernels can take (exact_kernels.hip)
    efast = ex.enabled && d.exact && pool.no > 0 && d.T <= kExactMaxT && (d.T - 1) * sc.us <= kExactMaxEntriesWide;
    if (CB > 1 && d.aligned) {
        LdsCarve cv = lds_carve(sc.Tcap, sc.Lcap, CB, sc.us);
        d.tmir = sc.tmir + (size_t)slot * sc.tmir_cap;
        d.gstart = (LDS uint16_t *)(smem + cv.o_gs);
        BatchView bv;
#ifdef SGUFP_TRACE
        bv.trace_on = 1;
#endif
#ifdef SGUFP_PROF
        bv.prof[0] = bv.prof[1] = 0;
#endif
        bv.vb = (LDS double *)(smem + cv.o_buf);
        bv.cring = (LDS double *)(smem + cv.o_ring);
        bv.tring = (LDS uint16_t *)(smem + cv.o_tring);
        bv.coef = (LDS double *)(smem + cv.o_bcoef);
        bv.w1 = smem + cv.o_w1;
        bv.ids = (LDS int32_t *)(smem + cv.o_ids);
        bv.wm = (LDS uint64_t *)(smem + cv.o_wm);
        bv.fm = bv.wm + (sc.Tcap + 63) / 64;
        bv.wsel = nullptr;
        bv.s2b = sc.s2b + (size_t)slot * sc.tail_cap * CB;
        bv.sm = sc.sm + (size_t)slot * sc.Tcap * CB;
        bv.xm = sc.xm + (size_t)slot * sc.Tcap * CB;
        build_stream(d, n_merged, CB * pool.ustride);   // tmir_cap = Ncap + Acap >= Nn + Amir
        const bool nxtry = ex.enabled && ex.nx && !ex.redo && !d.exact && pool.no >= ex.nx_min;
        if (d.stream) cut_loop_batched<CB>(net, d, sc, bv, pool, incumbent, st, efast, nxtry ? &ex : nullptr, slot, &nx_k0);
        else cut_loop_single(net, d, pool, incumbent, 0, st, efast);
#if defined(SGUFP_PROF) && defined(SGUFP_PHASES)
        st.ph[6] += bv.prof[0];
        st.ph[7] += bv.prof[1];
#endif
    } else {
        cut_loop_single(net, d, pool, incumbent, 0, st, efast);
    }
    st.stamp(6);
    if (st.status == kExactPending || st.status == kNxPending) {
        // hand-off: the root solution's slots for k_exact_root, then one pending entry and
        // this record's leaf passes (a single 64-bit atomic keeps the pass bases ascending
        // with the entry index, which k_exact_leaf's item search relies on); a non-exact DD
        // also records its tail's root layer k0 and starts its pruning position at 0
        GBL int32_t *rs = sc.rslot + (size_t)slot * sc.Lcap;
        for (int t = lane(); t < d.len; t += kWave) rs[t] = (int32_t)d.rslot[t];
        if (lane() == 0) {
            const uint32_t leaves = uni(d.nn[d.T - 1]);
            const unsigned long long passes = (leaves + (uint32_t)kLeafPass - 1) / (uint32_t)kLeafPass;
            const unsigned long long old = atomicAdd(ex.ctr, (1ull << 32) | passes);
            const int i = (int)(old >> 32);
            ex.pend_slot[i] = slot;
            ex.pend_base[i] = (uint32_t)(old & 0xFFFFFFFFull);
            ex.pidx[slot] = i;
            if (ex.pkind) {
                ex.pkind[i] = st.status == kNxPending ? nx_k0 : -1;
                ex.P[i] = 0;
                if (st.status == kNxPending) ex.nxlist[atomicAdd(&ex.ctr[12], 1ull)] = i;
            }
        }
    }
    if (st.status == kSuccess) {
        const GBL double *lrow = st.last_cut >= 0 ? pool.rows + (size_t)st.last_cut * pool.stride : nullptr;
        if (d.exact) {
            st.status = kNeedsSubproblem;
            int plen = dd_solution_path(net, d, lrow, out.path + (size_t)slot * sc.Lcap, rsol);
            if (lane() == 0) out.path_len[slot] = (uint16_t)plen;
        } else {
            int k = 3;
            while (k < d.T && uni(d.nalive[k]) != 1) k++;
            if (k >= d.T) {
                st.status = kErrCutset;
            } else {
                cut_layer = k;
                const uint32_t M = layer_single(d, k);
                if (uni(d.acnt[k])) {
                    const uint32_t aoff = uni(d.aoff[k]), acnt = uni(d.acnt[k]);
                    for (uint32_t base = 0; base < acnt; base += kWave) {
                        uint32_t a = base + lane();
                        nchild += wave_sum((a < acnt && (d.aflag[aoff + a] & kAlive)) ? 1u : 0u);
                    }
                } else {
                    nchild = (d.nflag[M] & kInAlive) ? 1u : 0u;
                }
            }
        }
    }
done:
    if (st.status == kPrunedFeasibility || st.status == kPrunedOptimality || st.status >= kErrRecord) {
        lb = DMIN;
        st.ub = DMIN;
    }
    if (lane() == 0) {
        out.status[slot] = st.status;
        out.exact[slot] = (uint8_t)d.exact;
        out.lb[slot] = lb;
        out.ub[slot] = st.ub;
        out.nchild[slot] = nchild;
        out.sol_need[slot] = nchild * (uint32_t)(d.len + cut_layer);
        out.dd_nodes[slot] = n_nodes;
        out.dd_arcs[slot] = n_arcs;
        out.dd_layers[slot] = (uint32_t)d.T + 1;
        out.sweeps[slot] = st.applied;
        out.redo[slot] = st.redo | (d.stream ? 0x80000000u : 0u) | ((d.Nn + d.Amir) << 8);
    }
    store_meta_layers(d, sc, slot, st.last_cut, st.status, cut_layer, st.ub);
    st.stamp(7);
#ifdef SGUFP_PHASES
    if (lane() == 0) {
        out.ticks[slot] = wall_clock64() - t_start;
        for (int k = 0; k < 8; k++) out.phase[(size_t)slot * 8 + k] = st.ph[k];
    }
#endif
}

// ------------------------------------------------------------------------------------
// Kernel 2: write cutset children (getCutset, DD.cpp:4179-4218) as frontier records.
__global__ void __launch_bounds__(kWave) k_emit_children(NetDev net, Scratch sc, BatchIn in, Pool pool,
                                                         BatchOut out, ChildOut co) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS uint8_t *smem = (LDS uint8_t *)smem_raw;
    const int slot = blockIdx.x;
    if (slot >= in.n) return;
    if (out.status[slot] != kSuccess || out.nchild[slot] == 0) return;
    DD d;
    dd_bind(d, smem, sc, slot);
    load_meta_layers(d, sc, slot);
    const GBL int32_t *meta = sc.meta + (size_t)slot * 8;
    const int last_cut = uni(meta[5]);
    const int k = uni(meta[7]);
    const double ub = sc.ubv[slot];
    const GBL double *row = last_cut >= 0 ? pool.rows + (size_t)last_cut * pool.stride : nullptr;
    const GBL int16_t *rsol = in.sol + in.sol_off[slot];
    const int gl = d.g + k;
    const int stride = d.len + k;
    const bool changed = net.changed[gl] != 0;
    uint32_t full = 0;
    if (changed) {
        int sl = net.set_len[net.layer_update[gl]];
        full = (sl >= 32) ? 0xFFFFFFFFu : ((1u << sl) - 1u);
    }
    const uint64_t cbase = co.child_off[slot];
    const uint64_t sbase = co.sol_base[slot];
    const uint32_t pnoff = uni(d.noff[k - 1]);
    const uint32_t M = layer_single(d, k);

    // enumerate the alive in-arcs of M in order: (parent, rank)
    const uint32_t acnt = uni(d.acnt[k]) ? uni(d.acnt[k]) : 1u;
    uint32_t child = 0;
    uint32_t cur_parent = 0xFFFFFFFFu;
    int plen = 0;
    for (uint32_t a = 0; a < acnt; a++) {
        uint32_t p, r;
        if (uni(d.acnt[k])) {
            if (!(d.aflag[uni(d.aoff[k]) + a] & kAlive)) continue;
            uint32_t t = d.atopo[uni(d.aoff[k]) + a];
            p = t & kParentMask;
            r = t >> kRankShift;
        } else {
            if (!(d.nflag[M] & kInAlive)) continue;
            uint32_t t = d.ntopo[M];
            p = t & kParentMask;
            r = t >> kRankShift;
        }
        if (p != cur_parent) {
            cur_parent = p;
            plen = dd_walk(net, d, pnoff + p, k - 1, row);
        }
        const uint64_t ci = cbase + child;
        const int64_t so = (int64_t)(sbase + (uint64_t)child * (uint64_t)stride);
        const int16_t dec = rank_value(net, d.g + k - 1, (int)r);
        for (int t = lane(); t < d.len; t += kWave) co.sol[so + t] = rsol[t];
        for (int t = lane(); t < plen; t += kWave) co.sol[so + d.len + t] = d.walk[plen - 1 - t];
        if (lane() == 0) {
            co.sol[so + d.len + plen] = dec;
            uint32_t pm = d.nmask[pnoff + p];
            co.gl[ci] = (uint16_t)gl;
            co.lb[ci] = DMIN;
            co.ub[ci] = ub;
            co.mask[ci] = changed ? full : ((r == 0) ? pm : (pm & ~(1u << r)));
            co.sol_off[ci] = so;
            co.sol_len[ci] = (uint16_t)(d.len + plen + 1);
        }
        child++;
        wave_lds_sync();
    }
}

// ------------------------------------------------------------------------------------
// Lazy terminal weights of exact DDs (ExactIO::lazy).  A flagged leaf's tw is the running
// min over the newest 64 x lazy O cuts of the exact phase (then over any refinement cuts
// since): an upper bound of its terminal weight.  The maximum over leaves only needs the
// exact value of the leaf that attains it: exact_argmax takes the first maximum, completes
// it over the remaining O cuts when it is flagged (exact_resolve), and repeats until the
// first maximum is exact -- every other leaf's true weight is <= its bound <= that value,
// and the ones before it are strictly below, so it is the reference's first maximum
// (DD.cpp:3975-3984).  Flagged leaves <= optimalLB are never completed: they cannot become
// the maximum of an unpruned DD (the incumbent only rises).

// Lanes = cuts of the blocks [ex.lazy, nblk) (newest-first positions), the leaf's path
// folded exactly as k_exact_leaf does; per lane a running min, then the wave min.  Zero
// bits: when the result is a zero above optimalLB, the first zero of the sequential order
// (the exact phase's cuts, newest first, then the refinement cuts tw has seen) decides.
__device__ void exact_resolve(const NetDev &net, DD &d, const ExactIO &ex, int i, uint32_t node, double incumbent) {
    const int T = d.T;
    // lane k holds layer k's (rank | in-alive << 7) and coefficient slot
    uint32_t info = 0;
    int slot = -1;
    {
        uint32_t nd = node;
        for (int k = T - 1; k >= 1; k--) {
            const uint32_t t = d.ntopo[nd];
            const uint32_t r = (t >> kRankShift) & 63u;
            const uint32_t b = r | ((d.nflag[nd] & kInAlive) ? 128u : 0u);
            if (lane() == k) {
                info = b;
                slot = r == 0 ? -1 : rank_slot(net, d, k, (int)r);
            }
            nd = uni(d.noff[k - 1]) + (t & kParentMask);
        }
    }
    const int nblk = (ex.no + kWave - 1) / kWave;
    const size_t os = (size_t)ex.ostride;
    auto value = [&](int s) -> double {
        const bool vc = s < ex.no;
        const int col = vc ? ex.no - 1 - s : 0;
        double c[kExactMaxT];
#pragma unroll
        for (int k = 1; k < kExactMaxT; k++) {
            c[k] = 0.0;
            if (k < T) {
                const int sl = __builtin_amdgcn_readlane(slot, k);
                if (sl >= 0 && vc) c[k] = ex.coefO[(size_t)sl * os + col];
            }
        }
        double v = vc ? ex.R[(size_t)i * os + s] : 0.0;
        sched_fence();
#pragma unroll
        for (int k = 1; k < kExactMaxT; k++) {
            if (k < T) {
                const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)info, k);
                v = !(b & 128u) ? DMIN : ((b & 63u) ? v + c[k] : v);
            }
        }
        return v;
    };
    double m = DMAX;
    for (int b = ex.lazy; b < nblk; b++) {
        const int s = b * kWave + lane();
        const double v = value(s);
        if (s < ex.no) m = (v < m) ? v : m;
    }
    m = wave_fmin(m);
    const double t0 = d.tw[node];
    double nv = (m < t0) ? m : t0;
    if (nv == 0.0 && nv > incumbent) {
        for (int b = 0; b < nblk; b++) {
            const int s = b * kWave + lane();
            const double v = value(s);
            const uint64_t hit = __ballot(s < ex.no && v == 0.0);
            if (hit) {
                nv = lane_get(v, (int)(__ffsll((unsigned long long)hit) - 1));
                break;
            }
        }
    }
    if (lane() == 0) {
        d.tw[node] = nv;
        d.nflag[node] &= (uint8_t)~kLazy;
        atomicAdd(&ex.ctr[4], 1ull);
        atomicAdd(&ex.ctr[5], (unsigned long long)(nblk - ex.lazy));
    }
    wave_mem_sync();
}

// first maximum over the alive leaves of an exact DD (vp_pick, first wins on ties), every
// flagged leaf that comes out on top above optimalLB completed first
__device__ VP exact_argmax(const NetDev &net, DD &d, const ExactIO &ex, int i, double incumbent) {
    const int last = d.T - 1;
    const uint32_t lo = uni(d.noff[last]), ln = uni(d.nn[last]);
    for (;;) {
        VP best{0.0, INT_MIN};
        for (uint32_t base = 0; base < ln; base += kWave) {
            const uint32_t k = base + lane();
            if (k < ln && (d.nflag[lo + k] & kAlive)) best = vp_pick(best, VP{d.tw[lo + k], prio_old((int)k)});
        }
        best = wave_vp(best);
        if (best.p == INT_MIN || !(best.v > incumbent) || i < 0) return best;
        const uint32_t node = lo + (uint32_t)(-best.p - 2);
        if (!(d.nflag[node] & kLazy)) return best;
        exact_resolve(net, d, ex, i, node, incumbent);
    }
}

// ------------------------------------------------------------------------------------
// Kernel 3: apply one freshly generated cut to exact DDs kept in their slots
// (the refinement loop of NodeExplorer.cpp:946-969).
__global__ void __launch_bounds__(kWave) k_refine(NetDev net, Scratch sc, BatchIn in, Pool pool, BatchOut out,
                                                  const int32_t *slots, const int32_t *cut_ids,
                                                  const uint8_t *cut_is_feas, int n, double incumbent, ExactIO ex) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS uint8_t *smem = (LDS uint8_t *)smem_raw;
    const int w = blockIdx.x;
    if (w >= n) return;
    const int slot = slots[w];
    if (out.status[slot] != kNeedsSubproblem) return;
    DD d;
    dd_bind(d, smem, sc, slot);
    load_meta_layers(d, sc, slot);
    const GBL int16_t *rsol = in.sol + in.sol_off[slot];
    for (int t = lane(); t < d.len; t += kWave) {
        int dec = rsol[t];
        int s = -1;
        if (dec != -1) {
            s = net.n_slots;
            if (dec >= 0 && dec < net.m) {
                int j = net.arc_head[dec];
                for (int q = net.slot_off[t]; q < net.slot_off[t + 1]; q++)
                    if (net.slot_head[q] == j) { s = q; break; }
            }
        }
        d.rslot[t] = (int16_t)s;
    }
    wave_lds_sync();
    const int id = cut_ids[w];
    const GBL double *row = pool.rows + (size_t)id * pool.stride;
    const double rv = root_fold(row, pool.rhs[id], d);
    dd_sweep(net, d, row, rv);
    int status = kNeedsSubproblem;
    double ub = sc.ubv[slot];
    if (lane() == 0) out.sweeps[slot] += 1u;
    // flagged (lazy) leaves: the batch's pending index of this record (-1: none flagged)
    // (ex.enabled: a launch without the exact phase leaves pidx of an earlier batch behind)
    const int pi = (ex.enabled && ex.lazy > 0 && d.exact) ? ex.pidx[slot] : -1;
    if (cut_is_feas[w]) {
        if (!dd_post_feasibility(net, d, row)) status = kPrunedFeasibility;
        else if (pi >= 0) exact_argmax(net, d, ex, pi, incumbent);   // the path below takes the first maximum
    } else {
        ub = dd_post_optimality(net, d, row, incumbent);
        if (pi >= 0 && ub > incumbent) {
            const VP best = exact_argmax(net, d, ex, pi, incumbent);
            ub = (best.p == INT_MIN) ? DMIN : smax(DMIN, best.v);
        }
        if (ub <= incumbent) status = kPrunedOptimality;
    }
    if (status == kNeedsSubproblem) {
        int plen = dd_solution_path(net, d, row, out.path + (size_t)slot * sc.Lcap, rsol);
        if (lane() == 0) out.path_len[slot] = (uint16_t)plen;
    }
    double lb = DMIN;
    if (status != kNeedsSubproblem) ub = DMIN;
    if (lane() == 0) {
        out.status[slot] = status;
        out.lb[slot] = lb;
        out.ub[slot] = ub;
    }
    store_meta_layers(d, sc, slot, id, status, 0, ub);
}

// ------------------------------------------------------------------------------------
// One DD at a time: the RelaxedDDNew surface (DD.h:797-808) behind the C++ API's
// Inavap::RelaxedDDNew.  A staged record is built with no cut applied (k_relax over an empty
// pool), then each call applies ONE cut to its resident DD -- exact or not, whatever its
// status -- exactly as the single-cut path of k_relax does (applyFeasibilityCut DD.cpp:3842-3930,
// applyOptimalityCut :3932-4023), and returns what the reference returns.  The cut's dense row
// is kept in the slot's own row (rows + slot * stride, meta last_cut = slot) so that
// getSolution / getCutset read the weights of the last cut applied (DD.cpp:3796-3840).
__global__ void __launch_bounds__(kWave) k_dd_apply(NetDev net, Scratch sc, BatchIn in, BatchOut out, int slot,
                                                    const double *rows, int stride, double rhs, int is_feas,
                                                    double optimal, double *value) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS uint8_t *smem = (LDS uint8_t *)smem_raw;
    DD d;
    dd_bind(d, smem, sc, slot);
    load_meta_layers(d, sc, slot);
    const GBL int32_t *meta = sc.meta + (size_t)slot * 8;
    const int status = uni(meta[6]), cut_layer = uni(meta[7]);
    const double ub = sc.ubv[slot];
    const GBL int16_t *rsol = in.sol + in.sol_off[slot];
    for (int t = lane(); t < d.len; t += kWave) {
        int dec = rsol[t];
        int s = -1;
        if (dec != -1) {
            s = net.n_slots;
            if (dec >= 0 && dec < net.m) {
                int j = net.arc_head[dec];
                for (int q = net.slot_off[t]; q < net.slot_off[t + 1]; q++)
                    if (net.slot_head[q] == j) { s = q; break; }
            }
        }
        d.rslot[t] = (int16_t)s;
    }
    wave_lds_sync();
    const GBL double *row = (const GBL double *)(rows + (size_t)slot * stride);
    dd_sweep(net, d, row, root_fold(row, rhs, d));
    double v;
    if (is_feas) v = dd_post_feasibility(net, d, row) ? 1.0 : 0.0;
    else v = dd_post_optimality(net, d, row, optimal);
    if (lane() == 0) {
        value[0] = v;
        out.sweeps[slot] += 1u;
    }
    store_meta_layers(d, sc, slot, slot, status, cut_layer, ub);
}

// getSolution (DD.cpp:3825-3840): argmax terminal weight, first-match walk of the last cut
__global__ void __launch_bounds__(kWave) k_dd_solution(NetDev net, Scratch sc, BatchIn in, BatchOut out, int slot,
                                                       const double *rows, int stride) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS uint8_t *smem = (LDS uint8_t *)smem_raw;
    DD d;
    dd_bind(d, smem, sc, slot);
    load_meta_layers(d, sc, slot);
    const int last = uni(sc.meta[(size_t)slot * 8 + 5]);
    const GBL double *row = last >= 0 ? (const GBL double *)(rows + (size_t)last * stride) : nullptr;
    const GBL int16_t *rsol = in.sol + in.sol_off[slot];
    const int plen = dd_solution_path(net, d, row, out.path + (size_t)slot * sc.Lcap, rsol);
    if (lane() == 0) out.path_len[slot] = (uint16_t)plen;
}

// getCutset(ub) (DD.cpp:4179-4218): the first width-1 layer at index >= 3 and the alive
// in-arcs of its node; k_emit_children writes them (status SUCCESS, nchild, cut layer)
__global__ void __launch_bounds__(kWave) k_dd_cutset(NetDev net, Scratch sc, BatchOut out, int slot, double ub) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS uint8_t *smem = (LDS uint8_t *)smem_raw;
    DD d;
    dd_bind(d, smem, sc, slot);
    load_meta_layers(d, sc, slot);
    const int last = uni(sc.meta[(size_t)slot * 8 + 5]);
    int status = kSuccess, k = 3;
    uint32_t nchild = 0;
    while (k < d.T && uni(d.nalive[k]) != 1) k++;
    if (d.exact || k >= d.T) {
        status = kErrCutset;   // a tree has no merged layer (the reference would run off its layers)
        k = 0;
    } else {
        const uint32_t M = layer_single(d, k);
        if (uni(d.acnt[k])) {
            const uint32_t aoff = uni(d.aoff[k]), acnt = uni(d.acnt[k]);
            for (uint32_t base = 0; base < acnt; base += kWave) {
                uint32_t a = base + lane();
                nchild += wave_sum((a < acnt && (d.aflag[aoff + a] & kAlive)) ? 1u : 0u);
            }
        } else {
            nchild = (d.nflag[M] & kInAlive) ? 1u : 0u;
        }
    }
    if (lane() == 0) {
        out.status[slot] = status;
        out.lb[slot] = DMIN;
        out.ub[slot] = ub;
        out.nchild[slot] = nchild;
        out.sol_need[slot] = nchild * (uint32_t)(d.len + k);
    }
    store_meta_layers(d, sc, slot, last, status, k, ub);
}

// ------------------------------------------------------------------------------------
// Kernel 4: end of the cut-parallel optimality phase of exact DDs (exact_kernels.hip):
// the terminal weights are final, so applyOptimalityCut's outcome is read off them --
// terminal state = first maximum over the alive leaves (DD.cpp:3975-3984); <= optimalLB:
// PRUNED_BY_OPTIMALITY_CUT, else ub = it and the argmax path (getSolution) -- and the DD is
// left as the reference's last cut (the oldest optimality cut) leaves it for k_refine.
__global__ void __launch_bounds__(kWave) k_exact_fin(NetDev net, Scratch sc, BatchIn in, Pool pool, BatchOut out,
                                                     ExactIO ex, double incumbent) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS uint8_t *smem = (LDS uint8_t *)smem_raw;
    const int i = blockIdx.x;
    if (i >= (int)(ex.ctr[0] >> 32)) return;
    const int slot = ex.pend_slot[i];
    if (out.status[slot] != kExactPending) return;   // a non-exact entry: k_nx_fin's
    DD d;
    dd_bind(d, smem, sc, slot);
    load_meta_layers(d, sc, slot);
    const VP best = exact_argmax(net, d, ex, ex.lazy > 0 ? i : -1, incumbent);
    const double term = (best.p == INT_MIN) ? DMIN : smax(DMIN, best.v);
    const int last_cut = pool.o_order[pool.no - 1];
    int status = kNeedsSubproblem;
    double ub = term;
    if (term <= incumbent) {
        status = kPrunedOptimality;
        ub = DMIN;
    } else {
        const GBL int16_t *rsol = in.sol + in.sol_off[slot];
        const int plen = dd_solution_path(net, d, pool.rows + (size_t)last_cut * pool.stride,
                                          out.path + (size_t)slot * sc.Lcap, rsol);
        if (lane() == 0) out.path_len[slot] = (uint16_t)plen;
    }
    if (lane() == 0) {
        out.status[slot] = status;
        out.lb[slot] = DMIN;
        out.ub[slot] = ub;
        out.sweeps[slot] += (uint32_t)pool.no;
    }
    store_meta_layers(d, sc, slot, last_cut, status, 0, ub);
}

// ------------------------------------------------------------------------------------
// Kernel 5: end of the cut-parallel optimality phase of non-exact DDs (kNxPending, see
// dd_device.hpp).  p = the first pool position where every leaf's running minimum is <=
// optimalLB (the terminal state, a maximum of those minima, only decreases, so the reference
// prunes there: applyOptimalityCut returns it and process stops, NodeExplorer.cpp:975-983).
// The width-1 pruning of DD.cpp:3986-4022 runs at a cut only when its terminal state is >
// optimalLB, i.e. at the positions before p; it removes an arc iff fl(fl(s + w) + gain) <=
// optimalLB - 0.01, i.e. (rounding is monotone) fl(xmin + fl(maxState - state2)) <= it for
// some width-1 layer.  k_nx_dag's per-cut gap G (a lower bound of min over the layers of
// xmin - state2 up to rounding) and the leaf passes' maxState decide conservatively: if no
// position before p can fire, no edit happened and the cut-parallel result is the
// reference's; otherwise the record is marked kNxFallback for k_relax's in-order re-run.
// Pruned: PRUNED_BY_OPTIMALITY_CUT at p.  Not pruned: ub = smin(last terminal state, ub)
// (the running smin over non-increasing states keeps the last), the DD's state2 set by the
// last (oldest) optimality cut's sweep for getCutset, and the cutset as k_relax's finish.
__device__ __forceinline__ double nx_unkey(unsigned long long k) {
    const unsigned long long b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    return __longlong_as_double((long long)b);
}

__global__ void __launch_bounds__(kWave) k_nx_fin(NetDev net, Scratch sc, BatchIn in, Pool pool, BatchOut out,
                                                  ExactIO ex, double incumbent) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS uint8_t *smem = (LDS uint8_t *)smem_raw;
    const int i = blockIdx.x;
    if (i >= (int)(ex.ctr[0] >> 32)) return;
    const int slot = ex.pend_slot[i];
    if (out.status[slot] != kNxPending) return;
    const int p = ex.P[i];
    const int first = ex.nxh[(size_t)slot * 4 + 3];   // k_relax applied positions [0, first) in order
    const int lim = p < pool.no ? p : pool.no;
    const double thresh = incumbent - 0.01;
    const size_t base = (size_t)i * ex.ostride;
    bool fire = false;
    for (int c0 = first; c0 < lim && !fire; c0 += kWave) {
        const int c = c0 + lane();
        bool f = false;
        if (c < lim) {
            const double gv = ex.G[base + c];
            const double M = nx_unkey(ex.MS[base + c]);
            f = !((gv + M) - 1e-12 * (fabs(M) + fabs(thresh) + 1.0) > thresh);   // NaN: may fire
        }
        fire = __ballot(f) != 0;
    }
    GBL int32_t *meta = sc.meta + (size_t)slot * 8;
    if (fire) {
        if (lane() == 0) {
            out.status[slot] = kNxFallback;
            ex.pkind[i] = kNxRouteFallback;   // sgufp_batch_routes: re-run in order by k_relax
            atomicAdd(&ex.ctr[7], 1ull);
        }
        return;
    }
    if (p < pool.no) {
        if (lane() == 0) {
            out.status[slot] = kPrunedOptimality;
            out.lb[slot] = DMIN;
            out.ub[slot] = DMIN;
            out.sweeps[slot] += (uint32_t)(p + 1 - first);
            meta[5] = pool.o_order[p];
            meta[6] = kPrunedOptimality;
            sc.ubv[slot] = DMIN;
        }
        return;
    }
    DD d;
    dd_bind(d, smem, sc, slot);
    load_meta_layers(d, sc, slot);
    const VP best = exact_argmax(net, d, ex, -1, incumbent);
    const double term = (best.p == INT_MIN) ? DMIN : smax(DMIN, best.v);
    double ub = smin(term, sc.ubv[slot]);
    int status = kSuccess, cut_layer = 0;
    uint32_t nchild = 0;
    const int last_cut = pool.o_order[pool.no - 1];
    if (ub <= incumbent) {
        status = kPrunedOptimality;   // not reached: p says some leaf stays above optimalLB
    } else {
        const GBL int32_t *rs = sc.rslot + (size_t)slot * sc.Lcap;
        for (int t = lane(); t < d.len; t += kWave) d.rslot[t] = (int16_t)rs[t];
        wave_lds_sync();
        const GBL double *row = pool.rows + (size_t)last_cut * pool.stride;
        dd_sweep(net, d, row, root_fold(row, pool.rhs[last_cut], d));
        int k = 3;
        while (k < d.T && uni(d.nalive[k]) != 1) k++;
        if (k >= d.T) {
            status = kErrCutset;
        } else {
            cut_layer = k;
            const uint32_t M = layer_single(d, k);
            if (uni(d.acnt[k])) {
                const uint32_t aoff = uni(d.aoff[k]), acnt = uni(d.acnt[k]);
                for (uint32_t b = 0; b < acnt; b += kWave) {
                    const uint32_t a = b + lane();
                    nchild += wave_sum((a < acnt && (d.aflag[aoff + a] & kAlive)) ? 1u : 0u);
                }
            } else {
                nchild = (d.nflag[M] & kInAlive) ? 1u : 0u;
            }
        }
    }
    if (status != kSuccess) ub = DMIN;
    if (lane() == 0) {
        out.status[slot] = status;
        out.lb[slot] = DMIN;
        out.ub[slot] = ub;
        out.nchild[slot] = nchild;
        out.sol_need[slot] = nchild * (uint32_t)(d.len + cut_layer);
        out.sweeps[slot] += (uint32_t)(pool.no - first);
    }
    store_meta_layers(d, sc, slot, last_cut, status, cut_layer, ub);
}

// ------------------------------------------------------------------------------------
// Exclusive scan of two u32 arrays into u64 offsets (n+1 entries), one 1024-thread block.
__global__ void __launch_bounds__(1024) k_scan2(const uint32_t *a, const uint32_t *b, int n, uint64_t *oa,
                                               uint64_t *ob) {
    __shared__ uint64_t sa[1024], sb[1024];
    const int t = threadIdx.x;
    const int per = (n + 1023) / 1024;
    const int lo = min(n, t * per), hi = min(n, lo + per);
    uint64_t xa = 0, xb = 0;
    for (int i = lo; i < hi; i++) { xa += a[i]; xb += b[i]; }
    sa[t] = xa; sb[t] = xb;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        uint64_t ya = (t >= d) ? sa[t - d] : 0, yb = (t >= d) ? sb[t - d] : 0;
        __syncthreads();
        sa[t] += ya; sb[t] += yb;
        __syncthreads();
    }
    uint64_t ra = sa[t] - xa, rb = sb[t] - xb;
    for (int i = lo; i < hi; i++) {
        oa[i] = ra; ob[i] = rb;
        ra += a[i]; rb += b[i];
    }
    if (t == 1023) { oa[n] = sa[1023]; ob[n] = sb[1023]; }
}

// ------------------------------------------------------------------------------------
// host-side launchers (called from capi.cpp)
size_t relax_lds_bytes(int Tcap, int Lcap, int cb, int us) { return lds_carve(Tcap, Lcap, cb, us).bytes; }

hipError_t launch_exact(const NetDev &net, const Scratch &sc, const ExactIO &ex, double incumbent, int cus,
                        hipStream_t st);

hipError_t launch_relax(const NetDev &net, const Scratch &sc, const BatchIn &in, const Pool &pool,
                        const BatchOut &out, double incumbent, int cb, const ExactIO &ex, int cus, hipStream_t st) {
    if (in.n <= 0) return hipSuccess;
    size_t lds = relax_lds_bytes(sc.Tcap, sc.Lcap, cb, sc.us);
    switch (cb) {
        case 4: hipLaunchKernelGGL(k_relax<4>, dim3(in.n), dim3(kWave), lds, st, net, sc, in, pool, out, incumbent, ex); break;
        case 8: hipLaunchKernelGGL(k_relax<8>, dim3(in.n), dim3(kWave), lds, st, net, sc, in, pool, out, incumbent, ex); break;
        case 16: hipLaunchKernelGGL(k_relax<16>, dim3(in.n), dim3(kWave), lds, st, net, sc, in, pool, out, incumbent, ex); break;
        default: hipLaunchKernelGGL(k_relax<1>, dim3(in.n), dim3(kWave), lds, st, net, sc, in, pool, out, incumbent, ex); break;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !ex.enabled || ex.no <= 0) return e;
    // exact DDs handed off by k_relax: root folds, terminal weights, outcome
    if ((e = launch_exact(net, sc, ex, incumbent, cus, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_exact_fin, dim3(in.n), dim3(kWave), relax_lds_bytes(sc.Tcap, sc.Lcap, 1, sc.us), st, net, sc, in,
                       pool, out, ex, incumbent);
    if ((e = hipGetLastError()) != hipSuccess || !ex.nx || !ex.pkind) return e;
    // non-exact DDs: outcome, then k_relax again over the records whose pruning might have fired
    hipLaunchKernelGGL(k_nx_fin, dim3(in.n), dim3(kWave), relax_lds_bytes(sc.Tcap, sc.Lcap, 1, sc.us), st, net, sc, in,
                       pool, out, ex, incumbent);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    ExactIO rx = ex;
    rx.redo = 1;
    switch (cb) {
        case 4: hipLaunchKernelGGL(k_relax<4>, dim3(in.n), dim3(kWave), lds, st, net, sc, in, pool, out, incumbent, rx); break;
        case 8: hipLaunchKernelGGL(k_relax<8>, dim3(in.n), dim3(kWave), lds, st, net, sc, in, pool, out, incumbent, rx); break;
        case 16: hipLaunchKernelGGL(k_relax<16>, dim3(in.n), dim3(kWave), lds, st, net, sc, in, pool, out, incumbent, rx); break;
        default: hipLaunchKernelGGL(k_relax<1>, dim3(in.n), dim3(kWave), lds, st, net, sc, in, pool, out, incumbent, rx); break;
    }
    return hipGetLastError();
}

hipError_t launch_scan(const uint32_t *a, const uint32_t *b, int n, uint64_t *oa, uint64_t *ob, hipStream_t st) {
    hipLaunchKernelGGL(k_scan2, dim3(1), dim3(1024), 0, st, a, b, n, oa, ob);
    return hipGetLastError();
}

hipError_t launch_emit(const NetDev &net, const Scratch &sc, const BatchIn &in, const Pool &pool,
                       const BatchOut &out, const ChildOut &co, hipStream_t st) {
    if (in.n <= 0) return hipSuccess;
    size_t lds = relax_lds_bytes(sc.Tcap, sc.Lcap, 1, sc.us);
    hipLaunchKernelGGL(k_emit_children, dim3(in.n), dim3(kWave), lds, st, net, sc, in, pool, out, co);
    return hipGetLastError();
}

bool relax_has_phases() {
#ifdef SGUFP_PHASES
    return true;
#else
    return false;
#endif
}

// RelaxedDDNew one DD at a time (k_dd_*): build without cuts, apply one cut, path, cutset
hipError_t launch_dd_build(const NetDev &net, const Scratch &sc, const BatchIn &in, const BatchOut &out, int stride,
                           hipStream_t st) {
    if (in.n <= 0) return hipSuccess;
    Pool none{};
    none.stride = stride;
    none.ustride = 1;
    ExactIO ex{};
    hipLaunchKernelGGL(k_relax<1>, dim3(in.n), dim3(kWave), relax_lds_bytes(sc.Tcap, sc.Lcap, 1, sc.us), st, net, sc,
                       in, none, out, DMIN, ex);
    return hipGetLastError();
}

hipError_t launch_dd_apply(const NetDev &net, const Scratch &sc, const BatchIn &in, const BatchOut &out, int slot,
                           const double *rows, int stride, double rhs, int is_feas, double optimal, double *value,
                           hipStream_t st) {
    hipLaunchKernelGGL(k_dd_apply, dim3(1), dim3(kWave), relax_lds_bytes(sc.Tcap, sc.Lcap, 1, sc.us), st, net, sc, in,
                       out, slot, rows, stride, rhs, is_feas, optimal, value);
    return hipGetLastError();
}

hipError_t launch_dd_solution(const NetDev &net, const Scratch &sc, const BatchIn &in, const BatchOut &out, int slot,
                              const double *rows, int stride, hipStream_t st) {
    hipLaunchKernelGGL(k_dd_solution, dim3(1), dim3(kWave), relax_lds_bytes(sc.Tcap, sc.Lcap, 1, sc.us), st, net, sc,
                       in, out, slot, rows, stride);
    return hipGetLastError();
}

hipError_t launch_dd_cutset(const NetDev &net, const Scratch &sc, const BatchOut &out, int slot, double ub,
                            hipStream_t st) {
    hipLaunchKernelGGL(k_dd_cutset, dim3(1), dim3(kWave), relax_lds_bytes(sc.Tcap, sc.Lcap, 1, sc.us), st, net, sc,
                       out, slot, ub);
    return hipGetLastError();
}

hipError_t launch_refine(const NetDev &net, const Scratch &sc, const BatchIn &in, const Pool &pool,
                         const BatchOut &out, const int32_t *slots, const int32_t *cut_ids,
                         const uint8_t *cut_is_feas, int n, double incumbent, const ExactIO &ex, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    size_t lds = relax_lds_bytes(sc.Tcap, sc.Lcap, 1, sc.us);
    hipLaunchKernelGGL(k_refine, dim3(n), dim3(kWave), lds, st, net, sc, in, pool, out, slots, cut_ids,
                       cut_is_feas, n, incumbent, ex);
    return hipGetLastError();
}

}  // namespace sgufp
