// wvg_heap.hpp -- the reference's bounded max-heap on the host, for the
// steps whose result depends on the heap's insertion history rather than on
// the distances alone: which member of a tie at the k-th distance survives,
// and in which order equal distances come out.
//
//   priorityqueue.Queue, NewMax       adapters/repos/db/priorityqueue/queue.go:42-50
//     Insert / insert                   :87-113   (sift up on strict less)
//     Pop / heapify                     :53-59, :131-147 (sift down, left first)
//   insertToHeap                      adapters/repos/db/vector/flat/index.go:497-506
//   extractHeap                       :508-520
//
// The device scans find every row such a heap can admit (wvg_replay.hip), so
// the host replays only those: a few thousand inserts per query.
#pragma once

#include <cstdint>
#include <vector>

namespace wvg {

struct GoItem {
    uint64_t id;
    float dist;
};

// priorityqueue.NewMax: less(i, j) = items[i].Dist > items[j].Dist.
struct GoMaxHeap {
    std::vector<GoItem> items;

    explicit GoMaxHeap(size_t capacity = 0) { items.reserve(capacity + 1); }
    size_t len() const { return items.size(); }
    const GoItem &top() const { return items[0]; }
    bool less(size_t i, size_t j) const { return items[i].dist > items[j].dist; }

    void insert(uint64_t id, float dist)  // queue.go:105-113
    {
        items.push_back(GoItem{id, dist});
        size_t i = items.size() - 1;
        while (i != 0 && less(i, (i - 1) / 2)) {
            std::swap(items[i], items[(i - 1) / 2]);
            i = (i - 1) / 2;
        }
    }
    void heapify(size_t i)  // queue.go:131-147 (its tail recursion as a loop)
    {
        for (;;) {
            const size_t left = 2 * i + 1, right = 2 * i + 2;
            size_t smallest = i;
            if (left < items.size() && less(left, i)) smallest = left;
            if (right < items.size() && less(right, smallest)) smallest = right;
            if (smallest == i) return;
            std::swap(items[i], items[smallest]);
            i = smallest;
        }
    }
    GoItem pop()  // queue.go:53-59
    {
        const GoItem out = items[0];
        items[0] = items.back();
        items.pop_back();
        heapify(0);
        return out;
    }
};

// flat.insertToHeap (V/flat/index.go:497-506).
inline void insert_to_heap(GoMaxHeap &h, size_t limit, uint64_t id, float dist)
{
    if (h.len() < limit) {
        h.insert(id, dist);
    } else if (h.top().dist > dist) {
        h.pop();
        h.insert(id, dist);
    }
}

// flat.extractHeap (V/flat/index.go:508-520): ascending by the pop order;
// returns the count written to ids / dists (capacity >= h.len()).
inline size_t extract_heap(GoMaxHeap &h, uint64_t *ids, float *dists)
{
    const size_t n = h.len();
    for (size_t i = n; i-- > 0;) {
        const GoItem it = h.pop();
        if (ids) ids[i] = it.id;
        if (dists) dists[i] = it.dist;
    }
    return n;
}

}  // namespace wvg
