// rt_records.cpp — host builders of the traversal records (rt_records.hpp).  Moved out of
// rt_device.hip's translation unit in round 6: host code only, compiled
// by the host compiler.
#include "rt_records.hpp"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <string>
#include <utility>

#include "rt_common.hpp"

namespace rt {
namespace {
constexpr uint32_t LEAF_BIT = kRecLeafBit;
constexpr uint32_t NO_REF = kRecNoRef;
}  // namespace

// Wide records for the camera rays' frustum traversal (traverse_frustum): an internal node's
// descendants D levels down in SearchBVH's push order, for the root and, in turn, every internal
// entry of a record; A = 2^D entries.  A leaf stands for itself and a child naming no valid
// triangle is skipped, as in the 4-ary records.  Records by their own index (an internal entry's
// ref is its record's), 8A floats: A x (x pair, y pair, z pair) | A refs (NO_REF pads) | unused.
// Exact for the reason the 4-ary records are (every internal box contains its children's,
// wide_ok).  The largest A in {32, 16, 8} (at most 2^dmax) whose DFS needs at most `cap` stack
// entries (FRUSTUM_STACK = 128: frog 32, bound 91; the c5 heightfield 32, bound 126); log2 = 2
// when none fits (the frustum traversal then takes the 4-ary records, wnode).
// cid: compact ids as rt_scene_create makes them (LEAF_BIT | slot, internal index, or NO_REF).
// (Leaf-pair entries, an internal node with two leaf children tested in one pop, measured no
// faster: c3 0.1517 vs 0.1517 ms, c5 48.2 vs 45.9; profiles/r04/exp/pairs_stack128_ab_*.log.)
// Valid leaves under each node (the greedy record rules' weights): a post-order walk from the
// root over the nodes rt_scene_create gave ids (cid: NO_REF for nodes naming no valid triangle).
std::vector<uint32_t> subtree_leaves(const rt_bvh_node* nodes, size_t NN, const uint32_t* cid) {
    std::vector<uint32_t> leaves(NN, 0u);
    std::vector<uint8_t> seen(NN, 0);  // each node expanded once (the tree is checked elsewhere)
    auto ref_of0 = [&](uint32_t n) -> uint32_t { return n == NO_REF || n >= NN ? NO_REF : cid[n]; };
    std::vector<std::pair<uint32_t, bool>> st{{0u, false}};
    while (!st.empty()) {
        auto [v, post] = st.back();
        st.pop_back();
        if (ref_of0(v) == NO_REF) continue;
        if (ref_of0(v) & LEAF_BIT) {
            leaves[v] = 1;
            continue;
        }
        if (!post) {
            if (seen[v]) continue;
            seen[v] = 1;
            st.push_back({v, true});
            for (uint32_t c : {nodes[v].left_idx, nodes[v].right_idx})
                if (c != NO_REF) st.push_back({c, false});
        } else {
            uint32_t sum = 0;
            for (uint32_t c : {nodes[v].left_idx, nodes[v].right_idx})
                if (c != NO_REF && ref_of0(c) != NO_REF) sum += leaves[c];
            leaves[v] = sum;
        }
    }
    return leaves;
}

FrustumRecords build_frustum_records(const rt_bvh_node* nodes, size_t NN, const uint32_t* cid,
                                            const rt_aabb* aabbs, int dmax, int cap) {
    FrustumRecords out;
    auto ref_of0 = [&](uint32_t n) -> uint32_t { return n == NO_REF ? NO_REF : cid[n]; };
    // RT_TUNE_RECORD_GREEDY: a record's entries are grown from its node's children by expanding,
    // in place (the DFS order stays the reference's), the internal entry of largest weight until
    // A entries: 2 (default) surface area x sqrt(valid leaves below), 1 surface area (3: x
    // log2(leaves + 1), 4: x leaves); 0: every path to the same depth.  Larger boxes are the ones
    // rays reach: c3 0.1412 vs 0.1452 ms, c5 41.0 vs 42.9 with the area (frog 3,416 records vs
    // 3,854, bound 94 vs 91; profiles/r05/exp/record_greedy_ab_c*.log); the leaf weight: c5
    // 39.3-39.9 vs 40.8-41.1, c3 within noise (record_rules_ab.log)
    const int greedy_rule = int(rt::tuning(RT_TUNE_RECORD_GREEDY, 2.0) + 0.5);
    const bool greedy = greedy_rule > 0;
    const std::vector<uint32_t> leaves = greedy_rule >= 2 ? subtree_leaves(nodes, NN, cid) : std::vector<uint32_t>();
    auto area = [&](uint32_t n) {
        const rt_aabb& b = aabbs[n];
        const double dx = std::max(0.0, double(b.max_corner.x) - b.min_corner.x);
        const double dy = std::max(0.0, double(b.max_corner.y) - b.min_corner.y);
        const double dz = std::max(0.0, double(b.max_corner.z) - b.min_corner.z);
        double a = dx * dy + dy * dz + dz * dx;
        if (greedy_rule == 2) a *= std::sqrt(double(leaves[n]));
        if (greedy_rule == 3) a *= std::log2(double(leaves[n]) + 1.0);
        if (greedy_rule == 4) a *= double(leaves[n]);
        return std::isfinite(a) ? a : 1e300;
    };
    for (int D = std::min(dmax, 5); D >= 3; --D) {
        const int A = 1 << D;
        auto expand = [&](auto&& self, uint32_t n, int d, uint32_t* e, int& k) -> void {
            if (ref_of0(n) == NO_REF) return;
            if (d == 0 || (ref_of0(n) & LEAF_BIT)) {
                e[k++] = n;
                return;
            }
            self(self, nodes[n].left_idx, d - 1, e, k);
            self(self, nodes[n].right_idx, d - 1, e, k);
        };
        std::vector<uint32_t> recs{0u};  // binary node of each record, breadth first
        std::vector<uint32_t> fid(NN, NO_REF);
        fid[0] = 0;
        std::vector<std::array<uint32_t, 32>> ents;
        std::vector<int> nent;
        for (size_t r = 0; r < recs.size(); ++r) {
            std::array<uint32_t, 32> e;
            int k = 0;
            if (greedy) {
                std::vector<uint32_t> fr;
                for (uint32_t c : {nodes[recs[r]].left_idx, nodes[recs[r]].right_idx})
                    if (ref_of0(c) != NO_REF) fr.push_back(c);
                while ((int)fr.size() < A) {
                    int best = -1;
                    double ba = -1.0;
                    for (int i = 0; i < (int)fr.size(); ++i) {
                        if (ref_of0(fr[i]) & LEAF_BIT) continue;
                        const double a = area(fr[i]);
                        if (a > ba) {
                            ba = a;
                            best = i;
                        }
                    }
                    if (best < 0) break;
                    std::vector<uint32_t> kids;
                    for (uint32_t c : {nodes[fr[best]].left_idx, nodes[fr[best]].right_idx})
                        if (ref_of0(c) != NO_REF) kids.push_back(c);
                    fr.erase(fr.begin() + best);
                    fr.insert(fr.begin() + best, kids.begin(), kids.end());
                }
                for (uint32_t n : fr) e[k++] = n;
            } else {
                expand(expand, nodes[recs[r]].left_idx, D - 1, e.data(), k);
                expand(expand, nodes[recs[r]].right_idx, D - 1, e.data(), k);
            }
            for (int i = 0; i < k; ++i)
                if (!(ref_of0(e[i]) & LEAF_BIT) && fid[e[i]] == NO_REF) {
                    fid[e[i]] = uint32_t(recs.size());
                    recs.push_back(e[i]);
                }
            ents.push_back(e);
            nent.push_back(k);
        }
        // DFS stack bound: entry i of a record is processed with entries 0..i-1 on the stack
        std::vector<int> SF(recs.size(), 0);
        for (size_t r = recs.size(); r-- > 0;) {
            int sf = nent[r];
            for (int i = 0; i < nent[r]; ++i)
                if (!(ref_of0(ents[r][i]) & LEAF_BIT)) sf = std::max(sf, i + SF[fid[ents[r][i]]]);
            SF[r] = sf;
        }
        if (SF[0] > cap) continue;
        out.rec.assign(size_t(8 * A) * recs.size(), 0.f);
        for (size_t r = 0; r < recs.size(); ++r) {
            float* w = &out.rec[size_t(8 * A) * r];
            for (int i = 0; i < A; ++i) {
                uint32_t wr = NO_REF;
                if (i < nent[r]) {
                    const uint32_t n = ents[r][i];
                    const rt_aabb& bb = aabbs[n];
                    const float v6[6] = {bb.min_corner.x, bb.max_corner.x, bb.min_corner.y,
                                         bb.max_corner.y, bb.min_corner.z, bb.max_corner.z};
                    std::memcpy(&w[6 * i], v6, sizeof(v6));
                    wr = (ref_of0(n) & LEAF_BIT) ? ref_of0(n) : fid[n];
                }
                std::memcpy(&w[6 * A + i], &wr, 4);
            }
        }
        out.log2 = D;
        out.bound = SF[0];
        out.nrec = recs.size();
        return out;
    }
    return out;
}

// The frustum records quantised (MODE_QR kernels: the big scenes, whose 1 KB records do not stay
// in the L2s): per record a grid over the union of its entries' boxes, origin o = the union's
// min and per axis a step h >= extent / 65534; entry bounds become 16-bit steps q_lo = the
// largest q with fma(q, h, o) <= min and q_hi = the smallest with fma(q, h, o) >= max, evaluated
// in float as the kernel does (fmaf, one rounding), so the dequantised box contains the entry's.
// The family test only decides what is pushed (leaves are tested exactly at pop), so looser
// boxes cost pops, never a different hit.  qent: A x (x lo | x hi << 16, y, z, ref) per record;
// qhdr: (o.x, o.y, o.z, h.x), (h.y, h.z, 0, 0).  False (no quantised records) when a bound is not
// finite, an extent exceeds 1e30 or a step would be subnormal.
bool build_quant_records(const FrustumRecords& fr, std::vector<uint32_t>& qent, std::vector<float>& qhdr) {
    const int A = 1 << fr.log2;
    qent.assign(size_t(4 * A) * fr.nrec, 0u);
    qhdr.assign(size_t(8) * fr.nrec, 0.f);
    for (size_t r = 0; r < fr.nrec; ++r) {
        const float* w = &fr.rec[size_t(8 * A) * r];
        uint32_t* qe = &qent[size_t(4 * A) * r];
        float* qh = &qhdr[8 * r];
        for (int a = 0; a < 3; ++a) {
            float lo = INFINITY, hi = -INFINITY;
            for (int i = 0; i < A; ++i) {
                uint32_t ref;
                std::memcpy(&ref, &w[6 * A + i], 4);
                if (ref == NO_REF) continue;
                lo = std::min(lo, w[6 * i + 2 * a]);
                hi = std::max(hi, w[6 * i + 2 * a + 1]);
            }
            if (lo > hi) lo = hi = 0.f;  // a record without entries (not built, kept total)
            if (!std::isfinite(lo) || !std::isfinite(hi) || double(hi) - double(lo) > 1e30) return false;
            float h = float((double(hi) - double(lo)) / 65534.0);
            if (double(h) * 65534.0 < double(hi) - double(lo)) h = std::nextafter(h, INFINITY);
            if (h != 0.f && !(h >= 1e-30f)) return false;
            (a == 0 ? qh[3] : qh[3 + a]) = h;
            qh[a] = lo;
            for (int i = 0; i < A; ++i) {
                uint32_t ref;
                std::memcpy(&ref, &w[6 * A + i], 4);
                if (ref == NO_REF) continue;
                const float mn = w[6 * i + 2 * a], mx = w[6 * i + 2 * a + 1];
                uint32_t ql = 0, qh16 = 0;
                if (h > 0.f) {
                    double fl = std::floor((double(mn) - double(lo)) / double(h));
                    double fh = std::ceil((double(mx) - double(lo)) / double(h));
                    ql = uint32_t(std::clamp(fl, 0.0, 65535.0));
                    qh16 = uint32_t(std::clamp(fh, 0.0, 65535.0));
                    while (ql > 0 && std::fmaf(float(ql), h, lo) > mn) --ql;
                    while (qh16 < 65535 && std::fmaf(float(qh16), h, lo) < mx) ++qh16;
                }
                if (std::fmaf(float(ql), h, lo) > mn || std::fmaf(float(qh16), h, lo) < mx) return false;
                qe[4 * i + a] = ql | (qh16 << 16);
            }
        }
        for (int i = 0; i < A; ++i) std::memcpy(&qe[4 * i + 3], &w[6 * A + i], 4);
    }
    return true;
}

}  // namespace rt

using rt::set_error;
using rt::kRecLeafBit;
using rt::kRecNoRef;

// Host-only view of build_frustum_records for the CPU tests (no device), with the ids as
// rt_scene_create makes them.  info: log2, bound, record count.  rec: copied when rec_cap
// (floats) suffices.
extern "C" int rt_debug_frustum_records(size_t P, const rt_bvh_node* nodes, const rt_aabb* aabbs, int max_log2,
                                        int stack_cap, int64_t* info, float* rec, size_t rec_cap) {
    if (P == 0 || !nodes || !aabbs || !info) return set_error(RT_ERR_ARG, "rt_debug_frustum_records: null argument");
    if (P > 0x3FFFFFFFull) return set_error(RT_ERR_UNSUPPORTED, "more than 2^30 triangles");
    const size_t NN = 2 * P - 1;
    // the caller's arrays are checked as rt_scene_create checks them: children in range and no
    // cycle reachable from the root (tests/test_host_fuzz.py)
    {
        std::vector<uint8_t> state(NN, 0);  // 0 new, 1 on the path, 2 done
        std::vector<std::pair<uint32_t, bool>> st{{0u, false}};
        while (!st.empty()) {
            auto [v, post] = st.back();
            st.pop_back();
            if (post) {
                state[v] = 2;
                continue;
            }
            if (state[v] == 1) return set_error(RT_ERR_ARG, "BVH contains a cycle");
            if (state[v] == 2) continue;
            state[v] = 1;
            st.push_back({v, true});
            const rt_bvh_node& nd = nodes[v];
            if (nd.object_idx != 0xFFFFFFFFu) continue;
            for (const uint32_t c : {nd.left_idx, nd.right_idx}) {
                if (c == kRecNoRef) continue;
                if (c >= NN) return set_error(RT_ERR_ARG, "BVH child index out of range");
                st.push_back({c, false});
            }
        }
    }
    std::vector<uint32_t> cid(NN, kRecNoRef);
    size_t n_int = 0, n_leaf = 0;
    for (size_t n = 0; n < NN; ++n) {
        if (nodes[n].object_idx == 0xFFFFFFFFu) cid[n] = uint32_t(n_int++);
        else if (nodes[n].object_idx < P) cid[n] = kRecLeafBit | uint32_t(n_leaf++);
    }
    if (nodes[0].object_idx != 0xFFFFFFFFu) {  // a leaf root: no records (rt_scene_create makes none)
        info[0] = 2;
        info[1] = 0;
        info[2] = 0;
        return RT_OK;
    }
    const rt::FrustumRecords fr = rt::build_frustum_records(nodes, NN, cid.data(), aabbs, std::clamp(max_log2, 2, 5), stack_cap);
    info[0] = fr.log2;
    info[1] = fr.bound;
    info[2] = (int64_t)fr.nrec;
    if (rec && rec_cap >= fr.rec.size() && !fr.rec.empty()) std::memcpy(rec, fr.rec.data(), fr.rec.size() * sizeof(float));
    return RT_OK;
}
