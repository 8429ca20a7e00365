"""CPU model of the fused MLP's transposed LDS image (csrc/hip/mlp_core.h Tile<MT>): the publish
step's 8-byte stores and the GEMM's A-operand fragments read back by ds_read_b64_tr_b16 (T mode,
AOp) must round-trip every element, for every tile height, with the chunk swizzle applied; the
swizzle must keep all three access kinds free of LDS bank conflicts (bank model of
MI355X_MICROARCH.md §LDS)."""
import pytest


def swz(MT, r):
    if MT == 1:
        return (r >> 2) & 1
    if MT == 2:
        return ((r >> 1) & 1) | (((r >> 3) & 1) << 1)
    if MT == 4:
        return (r & 3) | (((r >> 3) & 1) << 2)
    return (r & 3) | (((r ^ (r >> 3)) & 1) << 2) | ((r & 1) << 3)


def tix(MT, r, e):
    XS = MT * 16
    return r * XS + (((e >> 3) ^ swz(MT, r)) << 3) + (e & 7)


def tr16_read(img, addrs):
    """ds_read_b64_tr_b16 semantics: per 16-lane group, lane 4q + p supplies the address of row
    q, columns 4p..4p+3 of a 4 x 16 block; lane i receives column i of the 4 rows (row q in
    element q)."""
    out = [None] * 64
    for g in range(4):
        block = {}
        for i in range(16):
            q, p = i >> 2, i & 3
            a = addrs[16 * g + i]
            for t in range(4):
                block[(q, 4 * p + t)] = img.get(a + t)
        for i in range(16):
            out[16 * g + i] = [block[(q, i)] for q in range(4)]
    return out


@pytest.mark.parametrize("MT", [2, 4, 8])
def test_publish_then_transposed_a_fragments_round_trip(MT):
    BP = MT * 16
    K = 64
    img = {}
    # publish: lane (lr, lg) of tile n holds Y[mt*16 + 4 lg + r][c = 16 n + lr] for r < 4 and
    # stores them as 8 contiguous bytes at tix(c, mt*16 + 4 lg)
    for n in range(K // 16):
        for mt in range(MT):
            for lane in range(64):
                lr, lg = lane & 15, lane >> 4
                c = 16 * n + lr
                base = tix(MT, c, mt * 16 + 4 * lg)
                for r in range(4):
                    img[base + r] = ("y", mt * 16 + 4 * lg + r, c)
    for ks in range(K // 32):
        for mt in range(MT):
            halves = []
            for second in (0, 1):
                addrs = []
                for lane in range(64):
                    g, i = lane >> 4, lane & 15
                    q, p = i >> 2, i & 3
                    addrs.append(tix(MT, ks * 32 + 8 * g + q + 4 * second, mt * 16 + 4 * p))
                halves.append(tr16_read(img, addrs))
            for lane in range(64):
                lr, lg = lane & 15, lane >> 4
                frag = halves[0][lane] + halves[1][lane]
                # A[m = batch row mt*16 + lr][k = 32 ks + 8 lg + j]
                assert frag == [("y", mt * 16 + lr, ks * 32 + 8 * lg + j) for j in range(8)]


def _cycles(addrs, groups, dwords, mod):
    tot = 0
    for grp in groups:
        banks = {}
        for lane in grp:
            for w in range(dwords):
                dw = addrs[lane] // 4 + w
                banks.setdefault(dw % mod, set()).add(dw)
        tot += max(len(v) for v in banks.values())
    return tot


@pytest.mark.parametrize("MT", [2, 4, 8])
def test_swizzle_keeps_transposed_reads_conflict_free(MT):
    for ks in range(2):
        for mt in range(MT):
            for second in (0, 1):
                addrs = []
                for lane in range(64):
                    g, i = lane >> 4, lane & 15
                    addrs.append(2 * tix(MT, ks * 32 + 8 * g + (i >> 2) + 4 * second, mt * 16 + 4 * (i & 3)))
                # 2 x 32-lane halves, bank (a / 4) % 64, 2 dwords per lane: ideal 1 cycle per half
                assert _cycles(addrs, [range(32), range(32, 64)], 2, 64) == 2
