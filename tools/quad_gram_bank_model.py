#!/usr/bin/env python3
"""Bank model of the C2 simulator's per-update LDS traffic with the QuadGram moments (sde.hip), per the MI355X LDS
rules (MI355X_MICROARCH.md §LDS): ds_write_b128 in eight 8-lane groups, bank (a/4) mod 32; ds_read_b128 in four
16-lane groups and ds_read_b64 in two 32-lane groups, bank (a/4) mod 64. Rows are 8 floats, row r of the wave's
slot at dword f(r) = sum of w_i over the set bits i of r (linear layouts: w_i = 8 * 2^i is the unpadded slot).

For every padded linear layout and every choice of the two lane bits (a, b) that form a quad, it prints the LDS
cycles of one update: the two row writes, the two 1 KiB chunk reads of the coalesced store, and the quad's 12 Gram
reads (lane class c = its bits (a, b), pair k of a row read at pair (k + c) mod 4). The unpadded slot with the quad
on lane bits 3 and 4 is conflict-free for both kinds of read, which is the layout sde.hip uses.

    python tools/quad_gram_bank_model.py
"""
import itertools

B128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128 += [[l + 32 for l in g] for g in B128]
G32 = [range(0, 32), range(32, 64)]
W8 = [range(i, i + 8) for i in range(0, 64, 8)]


def cycles(addrs, groups, width, mod):
    tot = 0
    for g in groups:
        banks = {}
        for l in g:
            for j in range(width):
                banks.setdefault((addrs[l] + j) % mod, set()).add(addrs[l] + j)
        tot += max(len(v) for v in banks.values())
    return tot


def model(w, a, b):
    f = lambda row: sum(w[i] for i in range(6) if row >> i & 1)
    wr = sum(cycles([f(l) + 4 * h for l in range(64)], W8, 4, 32) for h in range(2))
    rd = sum(cycles([f((k * 64 + l) >> 1) + 4 * ((k * 64 + l) & 1) for l in range(64)], B128, 4, 64) for k in range(2))
    cls = lambda l: ((l >> a) & 1) | (((l >> b) & 1) << 1)
    rowr = lambda l, r: (l & ~((1 << a) | (1 << b))) | ((r & 1) << a) | ((r >> 1) << b)
    gr = sum(cycles([f(rowr(l, r)) + 2 * ((k + cls(l)) & 3) for l in range(64)], G32, 2, 64)
             for r in range(4) for k in range(3))
    return wr, rd, gr


def main():
    res = []
    for deltas in itertools.product((0, 8, 16, 24), repeat=6):
        w = [8 * (1 << i) + deltas[i] for i in range(6)]
        blocks = sorted(sum(w[i] for i in range(6) if r >> i & 1) for r in range(64))
        if any(b2 - b1 < 8 for b1, b2 in zip(blocks, blocks[1:])) or blocks[-1] + 8 > 1024:
            continue
        for a, b in itertools.combinations(range(6), 2):
            wr, rd, gr = model(w, a, b)
            res.append((rd + gr, wr, rd, gr, blocks[-1] + 8, (a, b), w))
    res.sort()
    print("read cycles, write, chunk reads (ideal 8), Gram reads (ideal 24), slot dwords, quad bits, row weights")
    for r in res[:8]:
        print(r)
    print("sde.hip layout (unpadded, quad bits 3, 4):", model([8, 16, 32, 64, 128, 256], 3, 4))
    print("naive quad (lane bits 0, 1):", model([8, 16, 32, 64, 128, 256], 0, 1))


if __name__ == "__main__":
    main()
