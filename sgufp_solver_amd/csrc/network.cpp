// Host-side flow network (see network.hpp for the reference citations).
#include "network.hpp"

#include <algorithm>
#include <fstream>
#include <sstream>

namespace sgufp {

bool Network::load_file(const std::string &path) {
    std::ifstream in(path);
    if (!in) { error = "cannot open " + path; return false; }
    int nn, mm, ss;
    if (!(in >> nn >> mm >> ss) || nn <= 0 || mm < 0 || ss <= 0) { error = "bad header"; return false; }
    std::vector<int32_t> t(mm), h(mm), l((size_t)mm * ss), u((size_t)mm * ss), r((size_t)mm * ss);
    for (int a = 0; a < mm; a++) {
        if (!(in >> t[a] >> h[a])) { error = "truncated arc list"; return false; }
        for (int s = 0; s < ss; s++)
            if (!(in >> l[(size_t)a * ss + s] >> u[(size_t)a * ss + s] >> r[(size_t)a * ss + s])) {
                error = "truncated scenario data"; return false;
            }
    }
    std::string tok;
    in >> tok;  // "Vbar"
    std::vector<int32_t> vb;
    int id;
    while (in >> id) vb.push_back(id);
    return load_arrays(nn, mm, ss, t.data(), h.data(), l.data(), u.data(), r.data(), (int)vb.size(), vb.data());
}

bool Network::load_arrays(int nn, int mm, int ss, const int32_t *tails, const int32_t *heads, const int32_t *lbs,
                          const int32_t *ubs, const int32_t *rewards, int n_vbar, const int32_t *vbar_ids) {
    n = nn; m = mm; S = ss;
    if (n > 65535) { error = "node ids must fit 16 bits (Cut.h:342-344 key packing)"; return false; }
    if (m > 32767) { error = "arc ids must fit int16 decisions (DD.h:424)"; return false; }
    tail.assign(tails, tails + m);
    head.assign(heads, heads + m);
    lb.assign(lbs, lbs + (size_t)m * S);
    ub.assign(ubs, ubs + (size_t)m * S);
    reward.assign(rewards, rewards + (size_t)m * S);
    out_arcs.assign(n, {});
    in_arcs.assign(n, {});
    for (int a = 0; a < m; a++) {
        if (tail[a] < 0 || tail[a] >= n || head[a] < 0 || head[a] >= n) { error = "arc endpoint out of range"; return false; }
        out_arcs[tail[a]].push_back(a);
        in_arcs[head[a]].push_back(a);
    }
    is_vbar.assign(n, 0);
    for (int k = 0; k < n_vbar; k++) {
        if (vbar_ids[k] < 0 || vbar_ids[k] >= n) { error = "V-bar id out of range"; return false; }
        is_vbar[vbar_ids[k]] = 1;
    }

    // V-bar order (shuffleVBarNodes): demand points first, then backward BFS layers.
    std::vector<int32_t> rest(vbar_ids, vbar_ids + n_vbar), order, frontier;
    std::vector<uint8_t> placed(n, 0);
    auto take = [&](int v) {
        if (placed[v]) return;
        if (std::find(rest.begin(), rest.end(), v) == rest.end()) return;
        placed[v] = 1;
        order.push_back(v);
    };
    for (int v = 0; v < n; v++)
        if (out_arcs[v].size() == 1 && head[out_arcs[v][0]] == n - 1) frontier.push_back(v);
    for (int v : frontier) take(v);
    auto drop_placed = [&]() {
        rest.erase(std::remove_if(rest.begin(), rest.end(), [&](int v) { return placed[v] != 0; }), rest.end());
    };
    drop_placed();
    int rounds = 0;
    while (!rest.empty()) {
        if (++rounds > n + 1) { error = "V-bar node not backward-reachable from a demand point (reference loops forever)"; return false; }
        std::vector<int32_t> parents;
        std::vector<uint8_t> seen(n, 0);
        for (int c : frontier)
            for (int a : in_arcs[c]) {
                int p = tail[a];
                if (!seen[p]) { seen[p] = 1; parents.push_back(p); }
            }
        for (int p : parents) take(p);
        drop_placed();
        frontier.swap(parents);
    }
    vbar = order;
    return finish();
}

bool Network::finish() {
    layer_arc.clear();
    state_update.clear();
    state_changed.clear();
    int i = 0;
    for (int q : vbar) {
        std::vector<int16_t> st;
        st.push_back(-1);
        for (int a : out_arcs[q]) st.push_back((int16_t)a);
        std::sort(st.begin(), st.end());
        st.erase(std::unique(st.begin(), st.end()), st.end());
        state_update.insert({i, st});
        bool first = true;
        for (int a : in_arcs[q]) {
            state_changed.push_back(first ? 1 : 0);
            first = false;
            layer_arc.push_back(a);
            i++;
        }
    }
    state_changed.push_back(0);
    L = (int)layer_arc.size();

    // distinct sets, update / universe per layer
    sets.clear();
    std::map<std::vector<int16_t>, int> set_id;
    layer_update.assign(L + 1, -1);
    layer_universe.assign(L + 1, -1);
    max_states = 0;
    for (auto &kv : state_update) {
        if (kv.first >= L) continue;  // buildTree only consults keys < totalLayers
        auto it = set_id.find(kv.second);
        int sid;
        if (it == set_id.end()) {
            sid = (int)sets.size();
            set_id[kv.second] = sid;
            sets.push_back(kv.second);
        } else sid = it->second;
        layer_update[kv.first] = sid;
        max_states = std::max(max_states, (int)kv.second.size());
    }
    if (max_states > kMaxStates) { error = "a V-bar node has more than 31 out-arcs (device state masks are 32 bits)"; return false; }
    int cur = -1;
    for (int l = 0; l <= L; l++) {
        if (layer_update[l] >= 0) cur = layer_update[l];
        layer_universe[l] = cur;
    }

    // coefficient slots: per layer (i,q) = processingOrder arc, the distinct heads j of q's out-arcs
    slot_off.assign(L + 1, 0);
    slot_head.clear();
    for (int l = 0; l < L; l++) {
        slot_off[l] = (int)slot_head.size();
        int q = head[layer_arc[l]];
        std::vector<int32_t> hs;
        for (int a : out_arcs[q])
            if (std::find(hs.begin(), hs.end(), head[a]) == hs.end()) hs.push_back(head[a]);
        for (int j : hs) slot_head.push_back(j);
    }
    slot_off[L] = (int)slot_head.size();
    n_slots = (int)slot_head.size();
    slot_tab.assign((size_t)std::max(L, 1) * kMaxStates, -1);
    for (int l = 0; l < L; l++) {
        int u = layer_universe[l];
        if (u < 0) continue;
        const auto &U = sets[u];
        for (size_t r = 0; r < U.size(); r++)
            slot_tab[(size_t)l * kMaxStates + r] = (U[r] == -1) ? -1 : slot_of(l, U[r]);
    }
    return true;
}

int Network::slot_of(int layer, int dec) const {
    if (dec == -1) return -1;
    if (dec < 0 || dec >= m || layer < 0 || layer >= L) return zero_slot();
    int j = head[dec];
    for (int s = slot_off[layer]; s < slot_off[layer + 1]; s++)
        if (slot_head[s] == j) return s;
    return zero_slot();
}

uint64_t Network::slot_key(int slot) const {
    // largest l with slot_off[l] <= slot; that layer is non-empty because slot_off[l+1] > slot
    int l = (int)(std::upper_bound(slot_off.begin(), slot_off.end(), slot) - slot_off.begin()) - 1;
    int a = layer_arc[l];
    uint64_t q = (uint64_t)head[a], i = (uint64_t)tail[a], j = (uint64_t)slot_head[slot];
    return q | (i << 16) | (j << 32);
}

}  // namespace sgufp
