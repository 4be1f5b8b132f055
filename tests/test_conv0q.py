"""conv 0's integer form (yolo.hip pack_conv0q, conv.hip conv0_kernel /
stem_kernel): the packer's balanced base-256 i8 digits reconstruct integers
Q = round(V / s) of V = w[rgb][ky][kx] / 255 at 2^-23 of each channel's
largest |V|; the kernel's per-digit sums (accumulators started at
128 sum D_i) are exact and below 2^24; and s (65536 T0 + (256 T1 + T2)) + b,
evaluated in f32 in the kernel's order, equals the f64 conv of x / 255 (BGR
window bytes, the reference's RGB order) to ~2^-22 of the output scale --
far inside the 1 bf16 ulp (+1e-6) the GPU layer test allows."""
import numpy as np

from rvs_amd.detect import weights


def _q_block(variant):
    from oracle import yolo_ref
    flat = weights.synthetic_weights(variant, seed=11)
    blob = weights.pack(variant, flat, "bf16")
    c0 = yolo_ref.conv_specs(variant)[0][0][2]
    qb = 3 * c0 * 64 + 20 * c0
    start = blob.size - ((qb + 255) & ~255)  # the block closes the blob (256-B aligned)
    blk = blob[start:start + qb]
    n = 3 * c0 * 64
    d = blk[:n].view(np.int8).reshape(3, c0, 64).astype(np.int64)
    s = blk[n:n + 4 * c0].view(np.float32)
    b = blk[n + 4 * c0:n + 8 * c0].view(np.float32)
    c = blk[n + 8 * c0:n + 20 * c0].view(np.int32).reshape(3, c0)
    w = flat[:c0 * 27].reshape(c0, 3, 3, 3).astype(np.float64)
    return c0, d, s, b, c, w, flat[c0 * 27:c0 * 28]


def test_conv0_digits_and_value():
    rng = np.random.default_rng(0)
    k = np.arange(64)
    pad = (k % 16 >= 9) | (k >= 48)
    for variant in (0, 2):
        c0, d, s, b, c, w, b_ref = _q_block(variant)
        np.testing.assert_array_equal(b, b_ref)
        assert (np.abs(d) <= 128).all() and (d <= 127).all()
        Q = d[0] * 65536 + d[1] * 256 + d[2]
        assert (Q[:, pad] == 0).all()
        np.testing.assert_array_equal(c, 128 * d.sum(2))
        V = np.zeros((c0, 64))
        for ky in range(3):
            for kx in range(3):
                for ch in range(3):
                    V[:, 16 * ky + 3 * kx + ch] = w[:, 2 - ch, ky, kx] / 255.0
        M = np.abs(V).max(1)
        assert (np.abs(Q * s[:, None].astype(np.float64) - V) <= (M * 2.0 ** -23)[:, None]).all()
        # random windows (some all-zero: the padding); zero-weight slots hold garbage
        x = rng.integers(0, 256, size=(4096, 64)).astype(np.int64)
        x[:64, ~pad] = 0
        T = []
        for i in range(3):
            acc = c[i][None, :] + (x - 128) @ d[i].T   # the MFMA: start + sum D (x - 128)
            np.testing.assert_array_equal(acc, x @ d[i].T)
            assert np.abs(acc).max() < 2 ** 24
            T.append(acc.astype(np.float32))
        # the kernel's combine: 256 T1 + T2 exactly in i32, then one fma
        t12 = (T[1].astype(np.int64) * 256 + T[2].astype(np.int64)).astype(np.float32)
        u = (T[0].astype(np.float64) * 65536 + t12.astype(np.float64)).astype(np.float32)
        got = (s[None, :] * u + b[None, :]).astype(np.float64)
        ref = x @ V.T + b.astype(np.float64)
        scale = np.abs(V).sum(1) * 255 + np.abs(b)
        assert (np.abs(got - ref) <= scale * 2.0 ** -21).all(), variant
