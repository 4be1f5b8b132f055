"""fp8 (OCP e4m3fn) plan, host side: the oracle's e4m3 rounding pinned
against torch's float8_e4m3fn cast and against the code table; the native
packer (rv_yolo_pack2, RV_YOLO_DTYPE_FP8) against the oracle's weight
quantiser (codes, scales and the documented packed layout); rv_fp8_scale
against the oracle's scale rule; and the oracle's fp8 graph end to end on a
small frame.  The device side (conv kernels on v_mfma_f32_16x16x32_fp8_fp8)
is test_fp8_gpu.py."""
import numpy as np
import torch

from oracle import yolo_ref as Y


def test_e4m3_table_and_rounding():
    v = Y.e4m3_table()
    assert v[0x7E] == 448.0 and v[0x08] == 2.0 ** -6 and v[0x01] == 2.0 ** -9
    codes = np.array([c for c in range(256) if c & 127 != 127], np.uint8)
    # every representable value maps to its own code (zeros: either sign)
    got = Y.e4m3_code(v[codes])
    assert ((got == codes) | ((codes & 127) == 0)).all()
    # midpoints round to the even code; anything past 448 saturates
    pos = v[:127]
    mid = (pos[:-1] + pos[1:]) / 2
    c = Y.e4m3_code(mid)
    assert (c % 2 == 0).all()
    assert (Y.e4m3_code(np.array([449.0, 1e9, -1e9])) == [0x7E, 0x7E, 0xFE]).all()


def test_e4m3_matches_torch_cast():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.normal(0, 1, 200000), rng.normal(0, 100, 200000),
                        rng.normal(0, 0.01, 200000)]).astype(np.float32)
    x = np.clip(x, -448, 448)
    ours = Y.e4m3_value(Y.e4m3_code(x))
    theirs = torch.from_numpy(x).to(torch.float8_e4m3fn).float().numpy()
    np.testing.assert_array_equal(ours, theirs)


def test_quant_fp8_equals_code_table():
    """quant_fp8 (torch's float8_e4m3fn cast after saturation) against the
    code-table rounding on every representable value, every midpoint (ties
    to even), the subnormal range, saturation and signed zeros, at several
    power-of-two buffer scales."""
    pos = Y.e4m3_table()[:127]
    mid = (pos[:-1] + pos[1:]) / 2
    rng = np.random.default_rng(3)
    x = np.concatenate([pos, -pos, mid, -mid, rng.normal(0, 60, 50000),
                        rng.uniform(-0.03, 0.03, 50000), [0.0, -0.0, 448.0, 470.0, 1e7, -1e7]])
    for s in (2.0 ** -6, 1.0, 2.0 ** 3):
        xs = (x * s).astype(np.float32)
        ref = Y.e4m3_value(Y.e4m3_code(xs.astype(np.float64) / s)) * s
        got = Y.quant_fp8(torch.from_numpy(xs), s).double().numpy()
        np.testing.assert_array_equal(got, ref)
        assert (np.signbit(got) == np.signbit(ref)).all()


def test_fp8_scale_rule_matches_native():
    from rvs_amd import _lib
    lib = _lib.load()
    for a in [0.0, 1e-9, 0.3, 1.0, 224.0, 448.0, 448.0001, 896.0, 3.7e4]:
        assert lib.rv_fp8_scale(a) == Y.fp8_scale(a), a
        if a > 0:
            s = Y.fp8_scale(a)
            assert 224.0 < a / s <= 448.0


def _layout(variant):
    """Byte offsets of the fp8 packed layout (include/rvhip.h): per conv,
    weights, f32 bias [Cout16], f32 scales [Cout16] (fp8 convs), each
    256-B aligned."""
    al = lambda x: (x + 255) & ~255  # noqa: E731
    specs, _ = Y.conv_specs(variant)
    off, out = 0, []
    for i, (n, ci, co, k, s, act) in enumerate(specs):
        cop = (co + 15) & ~15
        f8 = Y._fp8_conv(n)
        cip = ((ci + 63) & ~63) if f8 else ((ci + 31) & ~31)
        w_off = off
        off = al(off + (co * ci * k * k * 4 if i == 0 else cop * k * k * cip * (1 if f8 else 2)))
        b_off = off
        off = al(off + cop * 4)
        ws_off = None
        if f8:
            ws_off = off
            off = al(off + cop * 4)
        out.append((n, ci, co, k, f8, cip, w_off, b_off, ws_off))
    # conv 0's integer form (pack_conv0q) closes the blob: digits [3][C0][64]
    # i8, scales [C0] f32, biases [C0] f32, accumulator starts [3][C0] i32
    c0 = specs[0][2]
    return out, al(off + 3 * c0 * 64 + 20 * c0)


def test_fp8_packer_matches_oracle_quantiser():
    from rvs_amd.detect import weights
    for variant in (0, 2):
        flat = weights.synthetic_weights(variant, seed=3)
        blob = weights.pack(variant, flat, "fp8")
        lay, total = _layout(variant)
        assert blob.size == total
        off = 0
        for n, ci, co, k, f8, cip, w_off, b_off, ws_off in lay:
            nw = co * ci * k * k
            w = flat[off:off + nw].reshape(co, ci, k, k)
            b = flat[off + nw:off + nw + co]
            off += nw + co
            np.testing.assert_array_equal(blob[b_off:b_off + 4 * co].view(np.float32), b)
            if not f8:
                continue
            codes, sc, _ = Y.quant_weight_fp8(w)
            np.testing.assert_array_equal(blob[ws_off:ws_off + 4 * co].view(np.float32), sc, err_msg=n)
            got = blob[w_off:w_off + co * k * k * cip].reshape(co, k * k, cip)[:, :, :ci]
            want = codes.transpose(0, 2, 3, 1).reshape(co, k * k, ci)
            same = (got == want) | (((got & 127) == 0) & ((want & 127) == 0))
            assert same.all(), f"{n}: {int((~same).sum())} codes differ"
            assert (blob[w_off:w_off + co * k * k * cip].reshape(co, k * k, cip)[:, :, ci:] == 0).all()


def test_oracle_fp8_graph_runs_and_tracks_fp32():
    """The fp8 graph on a 128x128 frame with its own calibration: finite,
    and as close to the fp32 network as 3 mantissa bits allow.  Measured on
    the synthetic weights (YOLOv8n / m, 256x256): class-score error p99
    0.12 / 0.09 (bf16 storage: 0.011 / 0.006), box p99 14 / 16 px (bf16:
    0.9 / 1.2 px) -- the fp8 plan's accuracy cost, ~10x bf16's."""
    from rvs_amd.detect import weights
    from conftest import road_frame
    flat = weights.synthetic_weights(0, seed=1)
    x = Y.preprocess(road_frame(128, 128, seed=4)[None])
    sc = Y.fp8_calibration(0, flat, x)
    assert {"X0", "C2", "CAT14", "SP", "DA0", "model.2.m.0"} <= set(sc)
    ref = Y.YoloRef(0, flat).forward(x).numpy()
    q = Y.YoloRef(0, flat, quant="fp8", scales=sc).forward(x).numpy()
    assert np.isfinite(q).all()
    assert np.quantile(np.abs(q[:, 4:] - ref[:, 4:]), 0.99) < 0.2
    assert np.quantile(np.abs(q[:, :2] - ref[:, :2]), 0.99) < 24.0
