#!/usr/bin/env python3
"""CPU check of the operand maps planned for attn_fwd_v13: a
flash tile on v_mfma_f32_16x16x32_bf16 with the scores in registers and P
fed to the PV MFMA straight from them.  Pure numpy, no GPU; it simulates

  * the 16x16x32 MFMA lane layouts (cdna_hip_programming.md §3):
      A (16 rows x 32 k): lane l holds row l % 16, k = 8 (l // 16) + 0..7
      B (32 k x 16 cols): lane l holds col l % 16, k = 8 (l // 16) + 0..7
      C (16 x 16):        lane l holds col l % 16, rows 4 (l // 16) + 0..3
    (any permutation of k applied to A and B alike leaves the product
    unchanged -- that is what lets P go to the PV MFMA without a shuffle);
  * ds_read_b64_tr_b16 (T10): per 16-lane group, lane 4q+p supplies the
    address of row q, columns 4p..4p+3 of a 4 x 16 block; lane i receives
    column i, row q in element q;
  * the K / V tile image: 64 keys x 128 d bf16, plain 256-B rows, 16-B chunk
    c of row r at c ^ fsw(r), fsw(r) = ((r & 3) << 2) | ((r >> 2) & 3)
    (attn_fwd_v12's LDS-DMA image);

and checks, for one wave's 64 query rows and one 64-key tile:
  S^T = K Q^T as 4 key-blocks x 4 query-blocks of 16x16 (Q^T fragments as
  the B operand, K fragments read row-wise from the image as A);
  P^T for key pair kp = (kb 2kp, kb 2kp+1) packed per lane from its own S
  values; V^T fragments by two tr_b16 reads with the matching key order;
  O^T = V^T P^T as 8 d-blocks x 4 query-blocks;
  the epilogue pairing (lanes l and l ^ 16 swap halves so each lane stores
  16 contiguous bytes of one output row).
Exit status 0 when every product matches numpy to fp32 rounding.

    python tools/v13_layout_check.py            # operand maps
    python tools/v13_layout_check.py --banks    # LDS bank conflicts, swizzle search (~5 min)

Bank result (--banks): v12's fsw gives 2-way conflicts for both v13 reads
(the 16x16x32 K row read and the V^T tr_b16 read).  The linear swizzle
chunk ^ (8 r0 ^ 4 r1 ^ 2 r2) (r_b = bit b of the row; search key 0x248) is
conflict-free for both; see v13_sw below.
"""
from __future__ import annotations

import sys

import numpy as np

RNG = np.random.default_rng(0)
KT, D, QR = 64, 128, 64  # keys per tile, head dim, query rows per wave


def fsw(r: int) -> int:
    return ((r & 3) << 2) | ((r >> 2) & 3)


def image_store(tile: np.ndarray) -> np.ndarray:
    """[64 rows][128] -> swizzled byte image as a flat uint16 array."""
    img = np.zeros(KT * D, dtype=np.float32)
    for r in range(KT):
        for c in range(16):
            dst = r * 128 + 8 * (c ^ fsw(r))
            img[dst:dst + 8] = tile[r, 8 * c:8 * c + 8]
    return img


def img_addr(r: int, col: int) -> int:
    """Element index of (row r, column col) in the swizzled image."""
    c, w = divmod(col, 8)
    return r * 128 + 8 * (c ^ fsw(r)) + w


def mfma_16x16x32(a_lanes, b_lanes, c_lanes):
    """a_lanes / b_lanes: [64][8] per-lane operands, c_lanes [64][4]."""
    A = np.zeros((16, 32))
    B = np.zeros((32, 16))
    for l in range(64):
        for j in range(8):
            A[l % 16, 8 * (l // 16) + j] = a_lanes[l][j]
            B[8 * (l // 16) + j, l % 16] = b_lanes[l][j]
    Cm = A @ B
    out = np.array(c_lanes, dtype=np.float64).copy()
    for l in range(64):
        for i in range(4):
            out[l][i] += Cm[4 * (l // 16) + i, l % 16]
    return out


def tr_read(img: np.ndarray, row0, col0) -> list:
    """ds_read_b64_tr_b16 for the 64 lanes: row0(g), col0(g) give each
    16-lane group's 4 x 16 block; returns [64][4]."""
    out = [[0.0] * 4 for _ in range(64)]
    for g in range(4):
        # lane 4q+p of the group addresses row q, columns 4p..4p+3
        block = np.zeros((4, 16))
        for q in range(4):
            for p in range(4):
                for e in range(4):
                    block[q, 4 * p + e] = img[img_addr(row0(g) + q, col0(g) + 4 * p + e)]
        for i in range(16):
            out[16 * g + i] = [block[q, i] for q in range(4)]
    return out


def main() -> int:
    Q = RNG.standard_normal((QR, D)).astype(np.float32)
    K = RNG.standard_normal((KT, D)).astype(np.float32)
    V = RNG.standard_normal((KT, D)).astype(np.float32)
    kimg, vimg = image_store(K), image_store(V)
    bad = 0

    # ---- S^T(kb, qb) = K(kb) Q(qb)^T, chains over 4 d-steps of 32
    S = {}
    for kb in range(4):
        for qb in range(4):
            acc = [[0.0] * 4 for _ in range(64)]
            for ds in range(4):
                # A: K rows 16kb + l%16, d chunk 4ds + l//16 (one ds_read_b128)
                a = [[kimg[img_addr(16 * kb + l % 16, 8 * (4 * ds + l // 16) + j)] for j in range(8)]
                     for l in range(64)]
                # B: Q^T, lane holds query 16qb + l%16, d = 32ds + 8(l//16) + j
                b = [[Q[16 * qb + l % 16, 32 * ds + 8 * (l // 16) + j] for j in range(8)] for l in range(64)]
                acc = mfma_16x16x32(a, b, acc)
            S[kb, qb] = acc
            ref = K[16 * kb:16 * kb + 16] @ Q[16 * qb:16 * qb + 16].T  # [keys][queries]
            got = np.zeros((16, 16))
            for l in range(64):
                for i in range(4):
                    got[4 * (l // 16) + i, l % 16] = acc[l][i]
            err = np.abs(got - ref).max()
            if err > 1e-3:
                print(f"S^T({kb},{qb}) max err {err:.3e}")
                bad += 1

    # ---- P = S (no softmax here: the layout is what is checked), O^T =
    # sum_kp V^T(db, kp) P^T(qb, kp)
    O = {}
    for db in range(8):
        for qb in range(4):
            acc = [[0.0] * 4 for _ in range(64)]
            for kp in range(2):
                # P^T as B: lane's own S values, kb 2kp then kb 2kp+1 (keys
                # 32kp + 4g + i, then 32kp + 16 + 4g + i)
                b = [list(S[2 * kp, qb][l]) + list(S[2 * kp + 1, qb][l]) for l in range(64)]
                # V^T as A: lane i of group g gets d = 16db + i for those keys:
                # two tr reads, rows 32kp + 4g (+16), columns 16db .. 16db+15
                lo = tr_read(vimg, lambda g, kp=kp: 32 * kp + 4 * g, lambda g, db=db: 16 * db)
                hi = tr_read(vimg, lambda g, kp=kp: 32 * kp + 16 + 4 * g, lambda g, db=db: 16 * db)
                a = [lo[l] + hi[l] for l in range(64)]
                acc = mfma_16x16x32(a, b, acc)
            O[db, qb] = acc
    Sfull = (Q @ K.T)  # [queries][keys]
    Oref = Sfull @ V  # [queries][d]
    got = np.zeros((QR, D))
    for (db, qb), acc in O.items():
        for l in range(64):
            for i in range(4):
                got[16 * qb + l % 16, 16 * db + 4 * (l // 16) + i] = acc[l][i]
    err = np.abs(got - Oref).max() / max(1.0, np.abs(Oref).max())
    if err > 1e-5:
        print(f"O max rel err {err:.3e}")
        bad += 1

    # ---- epilogue pairing: lane (g, i) holds d 16db + 4g + 0..3 of query
    # 16qb + i.  Swapping with lane ^ 16 (v_permlane16_swap: groups 0 <-> 1,
    # 2 <-> 3) the even-db data of the odd group for the odd-db data of the
    # even group, each lane ends with 8 contiguous d (16 B) per db pair:
    # even g: d 16db + 8(g//2) .. +7 of the even db, odd g: of the odd db.
    for qb in range(4):
        for dbp in range(4):
            de, do = 2 * dbp, 2 * dbp + 1
            for l in range(64):
                g, i = l // 16, l % 16
                partner = l ^ 16
                if g % 2 == 0:
                    vals = list(O[de, qb][l]) + list(O[de, qb][partner])
                    db, d0 = de, 16 * de + 8 * (g // 2)
                else:
                    vals = list(O[do, qb][partner]) + list(O[do, qb][l])
                    db, d0 = do, 16 * do + 8 * (g // 2)
                ref = Oref[16 * qb + i, d0:d0 + 8]
                if np.abs(np.array(vals) - ref).max() > 1e-3 * max(1.0, np.abs(ref).max()):
                    print(f"epilogue qb {qb} db {db} lane {l}: mismatch")
                    bad += 1
                    break
    print("v13 layout check:", "ok" if not bad else f"{bad} failures")
    return 1 if bad else 0



# ---- LDS bank conflicts of v13's reads (MI355X_MICROARCH.md §LDS: bank =
# (byte address / 4) % 64; ds_read_b128 in four 16-lane groups, the
# ds_read_b64_tr_b16 in 32-lane halves), for the image swizzle sw(row)
B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
               list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
               list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]


def degree(addrs: dict, groups, nbytes: int) -> int:
    worst = 1
    for grp in groups:
        banks = {}
        for l in grp:
            for w in range(nbytes // 4):
                dword = addrs[l] // 4 + w
                banks.setdefault(dword % 64, set()).add(dword)
        worst = max(worst, max(len(s) for s in banks.values()))
    return worst


def conflicts(sw) -> tuple:
    """(worst K b128 degree, worst V tr_b16 degree) over every read of a tile."""
    addr = lambda r, chunk: r * 256 + 16 * (chunk ^ sw(r))  # noqa: E731
    kd = 1
    for kb in range(4):
        for ds in range(4):
            a = {l: addr(16 * kb + l % 16, 4 * ds + l // 16) for l in range(64)}
            kd = max(kd, degree(a, B128_GROUPS, 16))
    vd = 1
    halves = [list(range(32)), list(range(32, 64))]
    for kp in range(2):
        for hi in range(2):
            for db in range(8):
                a = {}
                for l in range(64):
                    g, q, p = l // 16, (l % 16) // 4, l % 4
                    r = 32 * kp + 16 * hi + 4 * g + q
                    col = 16 * db + 4 * p
                    a[l] = addr(r, col // 8) + 2 * (col % 8)
                vd = max(vd, degree(a, halves, 8))
    return kd, vd


def swizzle_search():
    """Linear swizzles chunk ^ (M . row_bits) over GF(2), M 4x4: the best
    (K degree, V degree) pairs."""
    best = {}
    for m in range(1 << 16):
        cols = [(m >> (4 * b)) & 15 for b in range(4)]  # image of row bit b
        def sw(r, cols=cols):
            v = 0
            for b in range(4):
                if (r >> b) & 1:
                    v ^= cols[b]
            return v
        best.setdefault(conflicts(sw), m)
    return best


def v13_sw(r: int) -> int:
    """The conflict-free swizzle the search found (0x248)."""
    return ((r & 1) << 3) | ((r & 2) << 1) | ((r & 4) >> 1)


if __name__ == "__main__" and "--banks" in sys.argv:
    print("v12 fsw:", conflicts(fsw), "v13_sw:", conflicts(v13_sw))
    res = swizzle_search()
    for key in sorted(res)[:6]:
        print(key, hex(res[key]))


if __name__ == "__main__" and "--banks" not in sys.argv:
    sys.exit(main())
