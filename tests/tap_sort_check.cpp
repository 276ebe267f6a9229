// tap_sort_check.cpp — audio-suite_amd/csrc/tap_sort.h against std::sort of the
// packed (offset, tap index) keys (the merge's former order), over random tap
// sets with heavy duplication, the UI's largest ER spans, offsets up to the
// 2^29-frame output limit, and the empty / single-tap cases.  Prints "bad N".
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
#include "tap_sort.h"

int main() {
    std::mt19937_64 rng(12345);
    int bad = 0, cases = 0;
    const uint32_t spans[] = {1, 2, 255, 256, 257, 28801, 65535, 65536, 1u << 20, (1u << 29) - 1};
    for (uint32_t span : spans)
        for (int m : {0, 1, 2, 7, 320, 2000})
            for (int rep = 0; rep < 20; ++rep) {
                std::vector<uint64_t> key(m), tmp(m), ref;
                uint32_t omax = 0;
                for (int k = 0; k < m; ++k) {
                    const uint32_t o = 1 + (uint32_t)(rng() % span);
                    key[k] = ((uint64_t)o << 32) | (uint32_t)k;
                    omax = std::max(omax, o);
                }
                ref = key;
                std::sort(ref.begin(), ref.end());
                const uint64_t* out = sort_taps_by_offset(key.data(), tmp.data(), m, omax);
                ++cases;
                if (!std::equal(ref.begin(), ref.end(), out)) ++bad;
            }
    printf("cases %d bad %d\n", cases, bad);
    return bad != 0;
}
