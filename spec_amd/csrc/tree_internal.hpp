// tree_internal.hpp — host-side pieces shared by tree.hip (layout, encoder) and tree_decode.hip
// (decoder): the layout of a spec_tree (include/spec_amd.h) with its device descriptor, the row
// kernels' launch shape, a grow-only device buffer.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "tree_core.hpp"

namespace spec {

unsigned row_grid(uint64_t rows); // blocks for a grid-stride pass over `rows` rows
bool is_scalar(int kind);

// The whole host-side description of a tree: the ABI layout + the device descriptor.
struct Layout {
    spec_tree_table tables[TREE_MAX_T];
    spec_tree_column cols[TREE_MAX_C];
    uint32_t nt = 0, nc = 0;
    TreeDesc desc;
};

// Builds the layout; false on an invalid tree (rules: include/spec_amd.h spec_tree).
bool build_layout(const spec_tree *tr, Layout &L);

// grow-only device buffer
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int reserve(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes, 256);
        if (hipMalloc(&p, want) != hipSuccess) return -1;
        cap = want;
        return 0;
    }
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

} // namespace spec
