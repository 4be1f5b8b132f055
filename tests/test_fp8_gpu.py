"""fp8 (OCP e4m3fn) plan of the YOLOv8 forward (RV_YOLO_DTYPE_FP8; BASELINE
configs[4]: "YOLOv8m 1280x1280 fp8 MFMA conv path").

  * Layer by layer: every conv launch is recomputed in float64 from the
    GPU's own fp8 input codes (decoded with the buffer's scale) and the
    oracle's fp8 weights (oracle/yolo_ref.py quant_weight_fp8, the same codes
    as the packer: test_fp8_cpu.py), then quantised like the kernel's
    epilogue (code of value / buffer scale, nearest even, saturated).  The
    GPU accumulates exact fp8 products in f32 and uses the hardware exp /
    reciprocal in SiLU, so a code may land on the neighbouring code when the
    exact value sits next to a rounding midpoint: every element within 1
    e4m3 ulp of the exact value, fewer than 1e-3 of them not on the nearest
    code.  bf16 features (the head's .1 stage) and f32 logits as in
    test_yolo_layers_gpu.py.  conv0 (f32 math) and SPPF (max over codes:
    exact) likewise.
  * Whole network against YoloRef(quant="fp8") -- the same quantisation
    (weights, per-buffer activation scales, bf16 head features).  The fp8
    MFMA does not accumulate exactly (tools/fp8_probe.hip,
    tools/fp8_scale_probe.hip: |err| up to 2^-11.8 of sum |products| within
    one 16x16x32 instruction, 2^-12.5 for the block-scaled 16x16x128), so
    ~0.3 % of each layer's codes land one step from the oracle's, and the
    plain He-normal synthetic network is chaotic in fp8 under such flips
    (the oracle itself keeps ~21-50 % of its detections at IoU >= 0.9 under
    a 3e-5..3e-4 relative perturbation before every rounding); YOLOv8m's
    synthetic weights carry a channel-coherent share that makes them
    ordered (95-97.5 %), so its network-level bar is 90 %.
  * Config 5 geometry (YOLOv8m, 1280x1280, fog frames): runs, the NMS on the
    GPU's own raw prediction is bit-exact against the restated NMS, and the
    fp8 detections track the bf16 plan's.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import road_frame
from oracle import cpu, yolo_ref as Y

pytestmark = pytest.mark.gpu


def bf16_to_f32(u16):
    return (u16.astype(np.uint32) << 16).view(np.float32)


def ulp_bf16(x):
    a = np.abs(x).astype(np.float32)
    e = np.floor(np.log2(np.maximum(a, 2.0 ** -126)))
    return 2.0 ** (e - 7)


def ulp_e4m3(q):
    """Spacing of e4m3 values around |q| (q in code units, |q| <= 448)."""
    e = np.floor(np.log2(np.maximum(np.abs(q), 2.0 ** -6)))
    return 2.0 ** (e - 3)


class Introspect8:
    def __init__(self, eng, B):
        from rvs_amd import _lib
        lib = _lib.load()
        torch.cuda.synchronize()
        self.B = B
        self.ws = eng.ws.cpu().numpy()
        n = lib.rv_yolo_trace(eng._h, None, 0)
        recs = np.zeros(n * 24, np.int32)
        lib.rv_yolo_trace(eng._h, recs.ctypes.data, n)
        self.recs = recs.reshape(n, 24)
        self.bufs = eng.buffers(B)
        self.scales = eng.act_scales

    def raw(self, buf):
        name, h, w, c, es, off = self.bufs[buf]
        n = self.B * h * w * c
        dt = {1: np.uint8, 2: np.uint16, 4: np.float32}[es]
        return self.ws[off:off + es * n].view(dt).reshape(self.B, h, w, c)

    def view(self, buf):
        """Stored values as float64."""
        es = self.bufs[buf][4]
        r = self.raw(buf)
        if es == 1:
            return Y.e4m3_value(r) * self.scales[buf]
        if es == 2:
            return bf16_to_f32(r).astype(np.float64)
        return r.astype(np.float64)


def _engine(variant, H, W, B, cuda, seed=1, imgsz=640, **kw):
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    flat = weights.synthetic_weights(variant, seed=seed)
    eng = YoloEngine(variant, flat, B, (H, W), device=cuda, dtype="fp8", imgsz=imgsz, **kw)
    return eng, flat


def _params(variant, flat):
    specs, _ = Y.conv_specs(variant)
    params, off = {}, 0
    for n, ci, co, k, s, act in specs:
        nw = co * ci * k * k
        params[n] = (flat[off:off + nw].reshape(co, ci, k, k), flat[off + nw:off + nw + co])
        off += nw + co
    return specs, params


def _check_fp8(name, got_codes, y, scale, yabs=None):
    """got_codes: the GPU's e4m3 codes; y: float64 exact values; yabs: the
    same conv over |x| and |w| (the magnitude the f32 accumulation carries).
    Returns (fraction of codes not the nearest, worst accumulation residue
    relative to yabs)."""
    q = np.clip(y / scale, -448.0, 448.0)
    got = Y.e4m3_value(got_codes)
    nearest = Y.e4m3_value(Y.e4m3_code(q))
    d = np.abs(got - q)
    # beyond the 1-ulp rounding window: what the accumulation must explain
    res = np.maximum(d - ulp_e4m3(q) * 1.0001, 0.0)
    rel = 0.0 if yabs is None else float((res / (yabs / scale + 1e-30)).max())
    bad = np.argwhere(res > (0.0 if yabs is None else ACC_REL * yabs / scale))
    for idx in bad[:12]:
        t = tuple(idx)
        print(f"  {name} {t}: exact {q[t]:.5f} got {got[t]:.5f} nearest {nearest[t]:.5f}"
              + ("" if yabs is None else f" |acc| {yabs[t] / scale:.3f}"))
    assert len(bad) == 0, f"{name}: {len(bad)} codes beyond 1 ulp + accumulation bound"
    off = float((got != nearest).mean())
    assert off < 5e-3, f"{name}: {off:.2e} of codes not the nearest"
    return off, rel


# f32 accumulation of the fp8 MFMA, relative to the sum of |products|
ACC_REL = 2.0 ** -12


def test_fp8_refuses_forward_without_scales(cuda):
    from rvs_amd._lib import RVError
    eng, _ = _engine(0, 640, 640, 1, cuda)
    lb = torch.zeros((1, eng.in_h, eng.in_w, 3), dtype=torch.uint8, device=cuda)
    with pytest.raises(RVError, match="scales"):
        eng.forward_raw(lb)
    with pytest.raises(RVError, match="power of two"):
        eng.set_act_scales([0.3] * len(eng.buffers(1)))
    eng.close()


@pytest.mark.parametrize("H,W,B,variant", [(640, 640, 1, 0), (1080, 1920, 2, 0),
                                            (640, 640, 1, 2)])
def test_fp8_every_conv_layerwise(cuda, H, W, B, variant):
    eng, flat = _engine(variant, H, W, B, cuda)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=30 + b)), 3)
                   for b in range(B)])
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda))
    eng.calibrate(lb)
    raw = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb, raw)
    ins = Introspect8(eng, B)
    specs, params = _params(variant, flat)
    assert len(ins.recs) == len(specs) - 1
    worst = []
    for r in ins.recs:
        (ci_, inb, incs, inco, Hin, Win, Ho, Wo, o0, o0cs, o0co, up0, o1, o1cs, o1co, up1,
         rb, rcs, rco, in_up, in2b, in2cs, in2co, split) = r.tolist()
        name, cin, cout, k, s, act = specs[ci_]
        w, b = params[name]
        if Y._fp8_conv(name):
            assert ins.bufs[inb][4] == 1, name
            wq = Y.quant_weight_fp8(w)[2]
        else:
            wq = Y._bf16(torch.from_numpy(w)).numpy()
        x = ins.view(inb)[..., inco:inco + cin]
        xt = torch.from_numpy(np.ascontiguousarray(x.transpose(0, 3, 1, 2)))
        y = F.conv2d(xt, torch.from_numpy(wq).double(), torch.from_numpy(b).double(), stride=s,
                     padding=k // 2)
        yabs = F.conv2d(xt.abs(), torch.from_numpy(np.abs(wq)).double(),
                        torch.from_numpy(np.abs(b)).double(), stride=s, padding=k // 2)
        yabs = yabs.numpy().transpose(0, 2, 3, 1)
        if act:
            y = F.silu(y)
        y = y.numpy().transpose(0, 2, 3, 1)
        if rb >= 0:
            y = y + ins.view(rb)[..., rco:rco + cout]
        for ob, oco, up in ((o0, o0co, up0), (o1, o1co, up1)):
            if ob < 0:
                continue
            es = ins.bufs[ob][4]
            g = ins.raw(ob)[..., oco:oco + cout]
            parts = [g[:, dy::2, dx::2] for dy in (0, 1) for dx in (0, 1)] if up else [g]
            for part in parts:
                if es == 1:
                    worst.append(_check_fp8(name, part, y, ins.scales[ob], yabs) + (name,))
                elif es == 2:
                    gv = bf16_to_f32(part).astype(np.float64)
                    rms = float(np.sqrt(np.mean(y ** 2))) + 1e-12
                    d = np.abs(gv - y)
                    assert float((d > ulp_bf16(y) * 1.01 + 1e-3 * rms).mean()) < 1e-4, name
                    assert (d <= 2 * ulp_bf16(y) + 1e-2 * rms).all(), name
                else:
                    rms = float(np.sqrt(np.mean(y ** 2))) + 1e-12
                    d = np.abs(part.astype(np.float64) - y)
                    assert (d <= 1e-4 * rms + 1e-5 * np.abs(y)).all(), f"{name}: f32 {d.max()}"
    print("layers with most off-nearest codes:", sorted(worst)[-3:])
    print("largest accumulation residue / sum|products|:", max(worst, key=lambda t: t[1]))
    # conv0 (f32 math from the u8 letterbox) into fp8 X0
    w, b = params["model.0"]
    x = torch.from_numpy(lb.cpu().numpy()[..., ::-1].transpose(0, 3, 1, 2).copy()).double() / 255
    y0 = F.silu(F.conv2d(x, torch.from_numpy(w).double(), torch.from_numpy(b).double(), stride=2,
                         padding=1)).numpy().transpose(0, 2, 3, 1)
    x0 = [i for i, bb in enumerate(ins.bufs) if bb[0] == "X0"][0]
    _check_fp8("model.0", ins.raw(x0), y0, ins.scales[x0], np.abs(y0) + 1e-6)
    # SPPF on codes: the 5/9/13 pools of the first quarter, exact
    sp = [i for i, bb in enumerate(ins.bufs) if bb[0] == "SP"][0]
    v = ins.view(sp)
    c = v.shape[-1] // 4
    t = torch.from_numpy(np.ascontiguousarray(v[..., :c].transpose(0, 3, 1, 2)))
    p1 = F.max_pool2d(t, 5, 1, 2)
    p2 = F.max_pool2d(p1, 5, 1, 2)
    p3 = F.max_pool2d(p2, 5, 1, 2)
    for j, p in enumerate((p1, p2, p3)):
        np.testing.assert_array_equal(v[..., (j + 1) * c:(j + 2) * c], p.numpy().transpose(0, 2, 3, 1))
    eng.close()


def _iou(a, b):
    x1, y1 = max(a[0], b[0]), max(a[1], b[1])
    x2, y2 = min(a[2], b[2]), min(a[3], b[3])
    inter = max(0, x2 - x1) * max(0, y2 - y1)
    u = (a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter
    return inter / u if u > 0 else 0


def _match(a, b, iou=0.9, min_score=0.27):
    """(matched, total): rows of `a` (score >= min_score) with a row of `b`
    of the same class at IoU >= iou."""
    tot = hit = 0
    for x, y in zip(a, b):
        for r in x:
            if r[4] < min_score:
                continue
            tot += 1
            hit += any(int(g[5]) == int(r[5]) and _iou(g, r) >= iou for g in y)
    return hit, tot


@pytest.mark.parametrize("H,W,variant", [(1080, 1920, 0), (640, 640, 2)])
def test_fp8_network_matches_fp8_oracle(cuda, H, W, variant):
    """Whole fp8 network against YoloRef(quant="fp8") with the GPU's own
    per-buffer scales, and against the fp32 network.

    YOLOv8m (config 5's model) runs weights with a channel-coherent share
    (tests/golden/make_yolo_scales.py SMOOTH[2] = 0.25): the fp8 oracle
    keeps 95-97.5 % of its own detections (class, IoU >= 0.9) under a 3e-5 /
    3e-4 relative perturbation of every activation before its rounding
    (tools/fp8_calib_study.py), so the GPU must match >= 90 % of the fp8
    oracle's detections at IoU >= 0.9 and vice versa, and >= 80 % of its
    detections must have an fp32 detection of the same class at IoU >= 0.5
    (fp8 rounding lowers scores: fp32 has ~1.5x the detections; measured
    on the CPU oracles 95 %).  YOLOv8n keeps the plain He-normal weights its
    bf16 bench and tests use; those are chaotic in fp8 (the oracle keeps 21 %
    of its detections under the same perturbation), so YOLOv8n fp8 is NOT a
    parity target: its loose bars (40 % at IoU 0.5, score p99.9 <= 0.15)
    only check that the plan runs and stays in the oracle's neighbourhood."""
    B, keep = 2, [0, 2, 3, 5, 7]
    eng, flat = _engine(variant, H, W, B, cuda, seed=0, classes_keep=keep)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=20 + b)), 3)
                   for b in range(B)])
    lbt = eng.letterbox(torch.from_numpy(fr).to(cuda))
    eng.calibrate(lbt)
    raw = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lbt, raw, candidates=False)
    got_raw = raw.cpu().numpy()
    dets, n = eng.run_letterboxed(lbt)
    dets, n = dets.cpu().numpy(), n.cpu().numpy()
    got = [dets[b, :n[b]] for b in range(B)]
    scales = {bb[0]: s for bb, s in zip(eng.buffers(B), eng.act_scales)}
    lb = Y.preprocess(lbt.cpu().numpy())
    ref_raw = Y.YoloRef(variant, flat, quant="fp8", scales=scales).forward(lb).numpy()
    ds = np.abs(got_raw[:, 4:] - ref_raw[:, 4:])
    db = np.abs(got_raw[:, :4] - ref_raw[:, :4])
    frac_box = float((db <= 1.0 + 0.01 * np.abs(ref_raw[:, :4])).mean())
    ref = Y.postprocess(ref_raw, (eng.in_h, eng.in_w), (H, W), classes_keep=keep)
    (h1, t1), (h2, t2) = _match(ref, got), _match(got, ref)
    fp32 = Y.postprocess(Y.YoloRef(variant, flat).forward(lb).numpy(), (eng.in_h, eng.in_w),
                         (H, W), classes_keep=keep)
    (f1, u1), (f2, u2) = _match(fp32, got), _match(got, fp32)
    (l1, n1), (l2, n2) = _match(ref, got, 0.5), _match(got, ref, 0.5)
    (k1, m1), (k2, m2) = _match(fp32, got, 0.5), _match(got, fp32, 0.5)
    print(f"fp8 v{variant} {H}x{W}: score |d| p99.9 {np.percentile(ds, 99.9):.4f} max "
          f"{ds.max():.4f}; box within 1px+1% {frac_box:.5f}; dets matched vs fp8 oracle "
          f"{h1}/{t1}, {h2}/{t2} (IoU 0.5: {l1}/{n1}, {l2}/{n2}); vs fp32 oracle {f1}/{u1}, "
          f"{f2}/{u2} (IoU 0.5: {k1}/{m1}, {k2}/{m2})")
    assert t1 > 0 and t2 > 0
    if variant == 2:
        assert h1 >= 0.9 * t1 and h2 >= 0.9 * t2
        assert k2 >= 0.8 * m2
    else:
        assert n1 > 0 and l1 >= 0.4 * n1 and l2 >= 0.4 * n2
        assert np.percentile(ds, 99.9) <= 0.15
    eng.close()


def test_fp8_config5_fog_1280(cuda):
    """configs[4] geometry: YOLOv8m at 1280x1280 on fog/rain frames made on the
    device, batch 4 (the bench runs 16).  NMS on the GPU's raw prediction is
    bit-exact against the restated NMS; fp8 detections track the bf16
    plan's (same weights, calibrated on this batch)."""
    from rvs_amd.augment import FogSynthesizer
    from rvs_amd.detect.yolo_hip import YoloEngine
    H = W = 1280
    B, keep = 4, [0, 2, 3, 5, 7]
    clean = torch.from_numpy(np.stack([road_frame(H, W, seed=70 + b) for b in range(B)])).to(cuda)
    frames = FogSynthesizer(level="medium", seed=5, rain_p=0.002, device=cuda,
                             filters=False).synthesize_batch(clean)
    eng, flat = _engine(2, H, W, B, cuda, seed=0, imgsz=1280, classes_keep=keep)
    assert eng.A == 33600
    lb = eng.letterbox(frames)
    eng.calibrate(lb)
    raw = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb, raw)
    dets, n = eng.nms_from_raw(raw)
    dets, n = dets.cpu().numpy(), n.cpu().numpy()
    ref = Y.postprocess(raw.cpu().numpy(), (H, W), (H, W), classes_keep=keep)
    for b in range(B):
        np.testing.assert_array_equal(dets[b, :n[b]], ref[b])
    d8, n8 = eng.run_letterboxed(lb)
    got8 = [r[:k] for r, k in zip(d8.cpu().numpy(), n8.cpu().numpy())]
    e16 = YoloEngine(2, flat, B, (H, W), imgsz=1280, device=cuda, classes_keep=keep)
    d16, n16 = e16.run_letterboxed(lb)
    got16 = [r[:k] for r, k in zip(d16.cpu().numpy(), n16.cpu().numpy())]
    (h1, t1), (h2, t2) = _match(got16, got8, 0.5), _match(got8, got16, 0.5)
    print(f"config5 fp8 vs bf16 plan (IoU 0.5): {h1}/{t1} bf16 dets matched, {h2}/{t2} fp8 "
          f"dets matched; IoU 0.9: {_match(got16, got8)}, {_match(got8, got16)}")
    # fp8 rounding lowers scores (the bf16 plan keeps more detections): most
    # fp8 detections must be bf16 ones (precision), and at least half of the
    # bf16 plan's detections must survive in fp8 (recall; fp32 keeps ~1.5x
    # the fp8 detections, so the floor sits below 1 / 1.5).  The YOLOv8m
    # fixture weights carry a channel-coherent share chosen for fp8
    # conditioning (weights.base_weights): no real checkpoint
    # pins this parity figure.
    assert t1 > 0 and t2 > 0 and h2 >= 0.8 * t2 and h1 >= 0.5 * t1
    eng.close()
    e16.close()
