"""CPU emulation of the fp32-block kernel's MFMA predict (SchedCondMfma,
lft_sweep_v2.hip): the LDS staging addresses, the v_mfma_f32_16x16x4_f32 operand and
result lane maps (cdna_hip_programming.md: lane l holds A[l & 15][k = l >> 4] and
B[k = l >> 4][l & 15]; D register r of lane l is D[4 (l >> 4) + r][l & 15]) and the
write-back, for one wave of 4 problems.  Returns the predicted A [Sigma' | m'] A~^T
rows as the kernel's registers hold them, to compare with the direct product.

    python tools/emu_mfma_predict.py        # prints the max relative difference
"""
import numpy as np

S, MM, ES = 13, 4, 4
SS = S * S
CHM = (SS * ES + 15) // 16
IMGM = CHM * 16                       # 688 B per problem image
NJM = (4 * CHM + 63) // 64
IMGM_W = NJM * 1024
CHB = (S * MM * ES + 15) // 16
IMGB_W = ((4 * CHB + 63) // 64) * 1024
OFF_A = IMGM_W
OFF_T = 3 * IMGM_W + IMGB_W
TILE_W = 4 * 272 * 8
WAVE_BYTES = OFF_T + TILE_W
ZB, MFB, MFP = 2880, 2880, 1152       # as the kernel's constants


def emulate(A, X):
    """A: [4, S, S] f32 blocks (the wave's images); X: [4, S, 16] rows of
    [Sigma' | m'] per problem (lane 13 = m'), lanes 14, 15 anything finite."""
    lds = np.zeros(WAVE_BYTES // 4, dtype=np.float32)
    rng = np.random.default_rng(0)
    lds[:] = rng.standard_normal(lds.size).astype(np.float32)  # garbage, finite
    zaddr = OFF_T
    lds[zaddr // 4: (zaddr + ZB) // 4] = 0.0                      # the zero area
    lds[(zaddr + MFB) // 4: (zaddr + MFB + 4 * MFP) // 4] = 0.0    # staging region
    for p in range(4):
        lds[(zaddr + 800 + p * IMGM) // 4] = 1.0                   # A~[13][13] per image offset
        lds[(OFF_A + p * IMGM) // 4: (OFF_A + p * IMGM) // 4 + SS] = A[p].reshape(-1)
    lanes = np.arange(64)
    c, g = lanes & 15, lanes >> 4
    mfb = zaddr + MFB
    mx_w = mfb + g * MFP + 4 * c
    mx_a = mfb + 4 * (17 * c + 4 * g)
    ms_w = mfb + 4 * (18 * c + 4 * g)
    ms_r = mfb + g * MFP + 4 * 18 * c
    ia = OFF_A  # problem 0's image
    ma_b, ma_a = [], []
    for kk in range(4):
        kx = 4 * g + kk
        inn = (c < S) & (kx < S)
        ma_b.append(np.where(inn, ia + 4 * (S * c + kx),
                             np.where((c == S) & (kx == S), zaddr + 800, zaddr)))
        ma_a.append(np.where(inn, ia + 4 * (S * c + kx), zaddr))
    rd = lambda addr: lds[addr // 4]  # noqa: E731
    # stage X rows (register i, lane (g, c)) as f32
    Xreg = np.stack([X[g, i, c] for i in range(S)])  # [S][64]
    for i in range(S):
        lds[(mx_w + 68 * i) // 4] = Xreg[i].astype(np.float32)

    def mfma(a_op, b_op, d):  # d [4 regs][64 lanes]
        A16 = np.zeros((16, 4)); B16 = np.zeros((4, 16))
        for l in range(64):
            A16[l & 15, l >> 4] = a_op[l]
            B16[l >> 4, l & 15] = b_op[l]
        D = np.zeros((16, 16))
        for l in range(64):
            for r in range(4):
                D[4 * (l >> 4) + r, l & 15] = d[r][l]
        D = D + A16 @ B16
        return np.array([[D[4 * (l >> 4) + r, l & 15] for l in range(64)] for r in range(4)])

    D1 = [np.zeros((4, 64)) for _ in range(4)]
    D2 = [np.zeros((4, 64)) for _ in range(4)]
    for kk in range(4):
        for p in range(4):
            D1[p] = mfma(rd(mx_a + p * MFP + 4 * kk), rd(ma_b[kk] + p * IMGM), D1[p])
    for kk in range(4):
        for p in range(4):
            D2[p] = mfma(rd(ma_a[kk] + p * IMGM), D1[p][kk], D2[p])
    for p in range(4):
        for r in range(4):
            lds[(ms_w + p * MFP + 4 * r) // 4] = D2[p][r].astype(np.float32)
    out = np.zeros((4, S, 16))
    for i in range(S):
        v = rd(ms_r + 4 * i)
        for l in range(64):
            out[l >> 4, i, l & 15] = v[l]
    return out


def main():
    rng = np.random.default_rng(7)
    A = (np.eye(S) + 0.1 * rng.standard_normal((4, S, S))).astype(np.float32)
    X = np.zeros((4, S, 16))
    for p in range(4):
        M = rng.standard_normal((S, S))
        X[p, :, :S] = M @ M.T / S
        X[p, :, S] = rng.standard_normal(S)
        X[p, :, S + 1:] = rng.standard_normal((S, 2))
    got = emulate(A, X)
    worst = 0.0
    for p in range(4):
        At = np.eye(S + 1)
        At[:S, :S] = A[p]
        ref = A[p].astype(float) @ X[p, :, :S + 1] @ At.T  # rows of A [Sigma' | m'] A~^T
        worst = max(worst, float(np.abs(got[p, :, :S + 1] - ref).max() / np.abs(ref).max()))
        assert np.all(got[p, :, S + 1:] == 0.0)
    print(f"max rel diff vs A [X | m] A~^T: {worst:.3e}")
    return worst


if __name__ == "__main__":
    main()
