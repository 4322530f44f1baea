// rt_records.hpp — host builders of the traversal records rt_scene_create uploads
// (rt_records.cpp): the camera rays' frustum records (2^D-ary expansions of the reference's
// binary tree), their quantised form, and the per-node leaf counts the
// greedy record rules weigh.  Host C++ only.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "rt_mi355x.h"

namespace rt {

// Compact node ids (cid): LEAF_BIT | leaf slot, internal index, or NO_REF (rt_device.hip's
// LEAF_BIT and NO_REF, which static_assert the same values).
constexpr uint32_t kRecLeafBit = 0x80000000u;
constexpr uint32_t kRecNoRef = 0xFFFFFFFFu;

struct FrustumRecords {
    int log2 = 2;
    int bound = 0;  // the DFS stack bound of the records (root record)
    size_t nrec = 0;
    std::vector<float> rec;
};

// Valid leaves under each node (post-order from the root; cid NO_REF: none).
std::vector<uint32_t> subtree_leaves(const rt_bvh_node* nodes, size_t NN, const uint32_t* cid);
// The largest-arity frustum records (2^3..2^dmax) whose DFS fits `cap` stack entries.
FrustumRecords build_frustum_records(const rt_bvh_node* nodes, size_t NN, const uint32_t* cid,
                                     const rt_aabb* aabbs, int dmax, int cap);
// The records quantised (16-bit grid steps per entry); false when they cannot be.
bool build_quant_records(const FrustumRecords& fr, std::vector<uint32_t>& qent, std::vector<float>& qhdr);

}  // namespace rt
