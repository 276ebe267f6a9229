// tap_sort.h — host: the early-reflection taps of one preset ordered by
// offset for the merge in msg_render_batch (MS:416-420 adds the taps in tap
// order; equal rounded offsets are merged in that order).  Header-only so
// tests/tap_sort_check.cpp compiles the same code.
//
// key[i] = (offset << 32) | tap index, built in increasing tap index.  A
// stable LSD radix sort on the offset bits (8-bit digits, as many passes as
// the largest offset needs: two for every UI setting, offsets < 2^16) gives the
// order std::sort gives on the whole key -- ties keep tap order -- in
// O(passes (m + 256)) instead of O(m log m) with a mispredicted branch per
// comparison: 320 taps 1.3 us vs 14 us for std::sort, which had made the merge
// the largest host cost of a short preset (the H48 point is host-bound).
#pragma once
#include <cstdint>
#include <utility>

// Sorts key[0, m) by key >> 32 (stable); tmp holds m entries.  Returns the
// array that holds the result (key or tmp).
inline uint64_t* sort_taps_by_offset(uint64_t* key, uint64_t* tmp, int m, uint32_t omax) {
    for (int shift = 32; shift < 64; shift += 8) {
        if (shift > 32 && (omax >> (shift - 32)) == 0) break;   // higher digits all zero
        uint32_t cnt[257] = {0};
        for (int i = 0; i < m; ++i) ++cnt[((key[i] >> shift) & 255u) + 1];
        for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
        for (int i = 0; i < m; ++i) tmp[cnt[(key[i] >> shift) & 255u]++] = key[i];
        std::swap(key, tmp);
    }
    return key;
}
