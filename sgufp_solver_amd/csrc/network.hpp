// Host-side flow network and the DD layer metadata derived from it.
//
// Semantics follow the reference loader Network::Network (/root/reference/Network.cpp:10-129)
// and shuffleVBarNodes (/root/reference/Network.cpp:132-186):
//   * text format "n m S", m lines "tail head (lb ub r)xS", token "Vbar", ids;
//   * V-bar order: demand points (single out-arc into n-1) first, then a backward BFS
//     keeping first occurrences (the reference keeps duplicate parents and grows
//     exponentially on deep networks; first-occurrence order is identical);
//   * one DD layer per incoming arc of each V-bar node, in that node's incoming-arc
//     order (processingOrder, Network.cpp:111-116);
//   * stateUpdateMap[first layer of q] = sorted(out-arcs(q) U {-1}), inserted with
//     map::insert semantics (an existing key is kept, Network.cpp:100-103);
//   * hasStateChanged[l] = 1 at each V-bar node's first layer, plus a trailing 0.
// On top of that it precomputes the dense, MI355X-side tables: per layer the state
// universe in force, and the "coefficient slots" a cut row is densified into.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace sgufp {

constexpr int kMaxStates = 32;          // state sets are u32 bitmasks on the device
constexpr int kRelaxedMaxWidth = 120;   // RELAXED_MAX_WIDTH (DD.h:732)

struct Network {
    int n = 0, m = 0, S = 0;
    std::vector<int32_t> tail, head;
    std::vector<int32_t> lb, ub, reward;          // [m * S], scenario-minor
    std::vector<std::vector<int32_t>> out_arcs, in_arcs;
    std::vector<uint8_t> is_vbar;
    std::vector<int32_t> vbar;                    // processing order of V-bar nodes
    std::vector<int32_t> layer_arc;               // processingOrder[l].second
    std::map<int, std::vector<int16_t>> state_update;   // stateUpdateMap
    std::vector<uint8_t> state_changed;           // hasStateChanged, size L+1
    int L = 0;                                    // totalLayers

    // ---- derived dense tables (device side) ----
    std::vector<std::vector<int16_t>> sets;       // distinct state sets (sorted, -1 first)
    std::vector<int32_t> layer_update;            // [L+1] set id applied at layer l, -1 if none
    std::vector<int32_t> layer_universe;          // [L+1] set id in force at layer l, -1 if none yet
    std::vector<int32_t> slot_off;                // [L+1] coefficient slots of layer l
    std::vector<int32_t> slot_head;               // [n_slots] head node j of each slot
    std::vector<int32_t> slot_tab;                // [L * kMaxStates] slot of (layer, state rank); -1 = no add (-1 decision / beyond set), zero_slot = absent key
    int n_slots = 0;
    int zero_slot() const { return n_slots; }
    int max_states = 0;

    // error text of the last failed load
    std::string error;

    bool load_file(const std::string &path);
    bool load_arrays(int n, int m, int S, const int32_t *tails, const int32_t *heads, const int32_t *lbs,
                     const int32_t *ubs, const int32_t *rewards, int n_vbar, const int32_t *vbar_ids);

    // coefficient slot of decision arc `dec` at coefficient layer `layer` (zero_slot if the
    // key (q_l, i_l, head(dec)) is not a slot of that layer; -1 for dec == -1)
    int slot_of(int layer, int dec) const;
    // Inavap::getKey(q, i, j) (Cut.h:342-344) of a slot
    uint64_t slot_key(int slot) const;

  private:
    bool finish();
};

}  // namespace sgufp
