// Device-side data of the restricted decision diagram (Inavap::RestrictedDDNew,
// /root/reference/DD.cpp:3090-3505), shared by rdd_kernels.hip and capi.cpp.
#pragma once

#include <cstdint>

#include "dd_device.hpp"

namespace sgufp {

constexpr int kRddMax = 128;   // widest restricted DD (the reference's callers use 128)

struct RddIO {
    int width;                          // max_width of RestrictedDDNew (<= kRddMax)
    int Tcap, Lcap;
    uint16_t SGUFP_GBL *topo;           // [B][Tcap][kRddMax] parent | rank << 7 of every node
    uint32_t SGUFP_GBL *cmask;          // [B][kRddMax] state masks of the first layer after the exact part
    uint32_t SGUFP_GBL *csm;            // [B][kRddMax] state masks of the exact cutset layer
    int16_t SGUFP_GBL *csdec;           // [B][kRddMax][Tcap] decisions of each cutset node (root to node)
    // per record
    int32_t SGUFP_GBL *status;          // kSuccess / kPrunedFeasibility / kPrunedOptimality / kErrRecord
    uint8_t SGUFP_GBL *exact;
    double SGUFP_GBL *lb;               // bound of the last optimality cut (node.lb if none)
    int16_t SGUFP_GBL *path;            // [B][Lcap] max path (getSolution), status kSuccess only
    uint16_t SGUFP_GBL *path_len;
    uint32_t SGUFP_GBL *cs_n;           // cutset nodes (0 for an exact tree)
    uint16_t SGUFP_GBL *cs_gl;          // their global layer
};

}  // namespace sgufp
