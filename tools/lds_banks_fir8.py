#!/usr/bin/env python3
"""LDS bank-conflict model of k_fir8's twiddle-table reads (fir4_fft.h / fir8_fft.h,
Fir4Geo<16384>: 1024 threads, radices 16 16 8 8) under the MI355X_MICROARCH.md model
of lds_banks.py (ds_read_b64: two groups of 32 lanes over 64 banks; a group costs one
extra cycle per extra distinct address on its busiest bank).  The two-level table
w_M^x = hi[x >> 7] * lo[x & 127] is read with x = e r (mod M) for power-of-two
multiples e, so the lo reads of a wave fall on few banks.  Prints extra cycles per
workgroup-transform for the current layout and for padded lo tables
phys(x) = x + (x >> s)."""
M = 16384; T = 1024

def cost(addrs):
    """addrs: 64 float2 indices (one per lane) of one ds_read_b64."""
    extra = 0
    for g in range(2):
        banks = {}
        for a in set(addrs[g * 32:(g + 1) * 32]):
            for d in (2 * a, 2 * a + 1):
                banks.setdefault(d % 64, set()).add(a)
        extra += max(len(v) for v in banks.values()) - 1
    return extra

def patterns():
    """(name, list of per-lane x lists): every fir_wM read of one transform pair."""
    out = []
    B8 = 3
    # forward pass 3 (R = 8, NS = 256, powers): e = 8 (j & 255), j = t, t + 1024
    for b in range(2):
        for w in range(T // 64):
            js = [w * 64 + l + b * T for l in range(64)]
            e = [8 * (j & 255) for j in js]
            out.append(("fwd p3 w", e)); out.append(("fwd p3 wB", [(x * B8) % M for x in e]))
    # forward pass 4 (R = 8, powers): e = js[h] (t; NB4 - t)
    for w in range(T // 64):
        for h in range(2):
            js = [(w * 64 + l) if h == 0 else (2 * T - (w * 64 + l)) % (2 * T) for l in range(64)]
            out.append(("fwd p4 w", js)); out.append(("fwd p4 wB", [(x * B8) % M for x in js]))
    # inverse pass 3' (R = 16, NS = 64, table): x = 16 (j & 63) r
    for w in range(T // 64):
        js = [w * 64 + l for l in range(64)]
        for r in range(1, 16):
            out.append(("inv p3 r%d" % r, [(16 * (j & 63) * r) % M for j in js]))
    # inverse pass 4' (R = 16, table): x = t r
    for w in range(T // 64):
        ts = [w * 64 + l for l in range(64)]
        for r in range(1, 16):
            out.append(("inv p4 r%d" % r, [(t * r) % M for t in ts]))
    return out

def evaluate(lo_pad, hi_pad=None):
    tot = {}
    for name, xs in patterns():
        lo = [(x & 127) + ((x & 127) >> lo_pad if lo_pad else 0) for x in xs]
        hi = [1024 + (x >> 7) + (((x >> 7) >> hi_pad) if hi_pad else 0) for x in xs]
        key = name.split(" r")[0].split(" w")[0]
        tot[key] = tot.get(key, 0) + cost(lo) + cost(hi)
    return tot

if __name__ == "__main__":
    for s in (None, 5, 4, 3, 2):
        t = evaluate(s)
        print("lo pad", s, sum(t.values()), t)
    for s in (4, 3):
        for hs in (5, 4, 3):
            t = evaluate(s, hs)
            print("lo pad", s, "hi pad", hs, sum(t.values()), t)
