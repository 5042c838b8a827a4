"""LDS bank model of the direct conv kernels' MFMA operand reads (csrc/direct.h).

Lane groups and bank rule from MI355X_MICROARCH.md (LDS): ds_read_b128 serves
four 16-lane groups on 64 banks, ds_read_b64 two 32-lane groups.  For each
layer configuration it prints the LDS cycles of one A (patch) and B (weight)
read per wave against the conflict-free minimum, over row-stride paddings,
then searches (pixel stride, row padding) pairs.  RS = 32 (mod 64) came out
conflict-free for every layer and the PMC pass confirmed it
(profiles/r01_lds_conflicts.txt).

Usage: python tools/lds_banks.py
"""
G128 = [list(range(0,4))+list(range(12,16))+list(range(20,28)),
        list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128 = G128 + [[x+32 for x in g] for g in G128]
G64 = [list(range(32)), list(range(32, 64))]
def cycles(addrs, width):
    groups = G128 if width == 4 else G64
    tot = 0
    for g in groups:
        banks = {}
        for l in g:
            a = addrs[l]
            for k in range(width):
                banks.setdefault((a + k) % 64, set()).add((a + k))
        tot += max(len(v) for v in banks.values())
    return tot, len(groups)
def cfg(CP, N, KS, TY, TX, WM, WN, rs_pad=0, cs=None, cw=None):
    V = 4 if CP >= 8 else CP // 2
    CS = cs if cs else (CP + 4 if CP >= 8 else CP)
    PW = TX + KS - 1
    RS = PW * CS + (0 if CP >= 8 else 2) + rs_pad
    CW = cw if cw else (CP + 4 if CP >= 8 else CP)
    TM = TY * TX // WM // 32; TN = N // WN // 32
    ra = []; rb = []
    for wmi in range(WM):
        for i in range(TM):
            ad = []
            for l in range(64):
                m = wmi * TM * 32 + 32 * i + (l & 31); h = l >> 5
                win = m >> 2; dy = (m >> 1) & 1; dx = m & 1
                wy, wx = win // (TX // 2), win % (TX // 2)
                ad.append((2 * wy + dy) * RS + (2 * wx + dx) * CS + h * V)
            ra.append(cycles(ad, V))
    for wni in range(WN):
        for j in range(TN):
            ad = [(wni * TN * 32 + 32 * j + (l & 31)) * CW + (l >> 5) * V for l in range(64)]
            rb.append(cycles(ad, V))
    return RS, ra, rb
import sys
confs = {"conv1f": (4,32,7,16,16,4,1), "conv2f": (32,64,5,8,16,4,2), "conv3f": (64,64,3,8,8,2,2),
         "conv3d": (64,64,3,4,8,1,2), "conv2d": (64,32,5,8,16,4,1)}
for k, c in confs.items():
    for pad in (0, 4, 8, 12, 16, 20, 24, 28, 32):
        RS, ra, rb = cfg(*c, rs_pad=pad)
        print(k, "pad", pad, "RS", RS, "A", ra[:4], "B", rb[:2])
print("---- search")
for k in ("conv3f", "conv3d", "conv2f", "conv2d"):
    c = confs[k]
    best = []
    for cs in (68, 72, 76, 80):
        for pad in range(0, 64, 4):
            RS, ra, rb = cfg(*c, rs_pad=pad, cs=cs)
            best.append((max(x[0] for x in ra), cs, pad, RS))
    best.sort()
    print(k, best[:4])
for cw in (4, 6, 10, 12):
    RS, ra, rb = cfg(*confs["conv1f"], cw=cw)
    print("conv1 cw", cw, rb)
