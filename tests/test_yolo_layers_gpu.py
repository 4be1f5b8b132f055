"""Layer-wise parity of the YOLOv8 HIP forward.

Every conv launch of a forward is re-computed on the CPU from the GPU's own
input activations (read back from the workspace; no buffer is reused inside
a forward), with the same bf16 weights, in float64, then rounded like the
kernel's epilogue.  This isolates each kernel from the error amplification of
the full network (see test_detect_gpu.py).

Tolerance per output element: |gpu - ref| <= 1 bf16 ulp of |ref| (+1e-3 of
the layer RMS for cancellation near zero); fewer than 1e-4 of the elements
may exceed that, and none by more than 2 ulp + 1e-2 RMS.  f32 head logits:
|d| <= 1e-4 * RMS + 1e-5 |ref|.  SPPF pooling and the concat / upsample
copies: exact.  Decode (DFL + dist2bbox + sigmoid) from the GPU's own head
logits: |d| <= 1e-4 px / 1e-6.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import road_frame
from oracle import cpu, yolo_ref

pytestmark = pytest.mark.gpu


def bf16_to_f32(u16):
    return (u16.astype(np.uint32) << 16).view(np.float32)


def round_bf16(x):
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(torch.bfloat16).float().numpy()


def ulp_bf16(x):
    a = np.abs(x).astype(np.float32)
    e = np.floor(np.log2(np.maximum(a, 2.0 ** -126)))
    return 2.0 ** (e - 7)


class Introspect:
    def __init__(self, eng, B):
        from rvs_amd import _lib
        self.lib = _lib.load()
        self.eng = eng
        self.B = B
        torch.cuda.synchronize()
        self.ws = eng.ws.cpu().numpy()
        n = self.lib.rv_yolo_trace(eng._h, None, 0)
        recs = np.zeros(n * 24, np.int32)
        self.lib.rv_yolo_trace(eng._h, recs.ctypes.data, n)
        self.recs = recs.reshape(n, 24)
        self.bufs = []
        for i in range(self.lib.rv_yolo_num_buffers(eng._h)):
            info = (ctypes.c_int * 4)()
            off = ctypes.c_size_t()
            self.lib.rv_yolo_buffer_info(eng._h, B, i, info, ctypes.byref(off))
            self.bufs.append((info[0], info[1], info[2], info[3], off.value))

    def raw_u16(self, buf, cs=None):
        h, w, c, f32, off = self.bufs[buf]
        c = cs or c
        n = self.B * h * w * c
        return self.ws[off:off + 2 * n].view(np.uint16).reshape(self.B, h, w, c)

    def view(self, buf, cs=None):
        """`cs`: the channel stride a forward actually used (a fused C2f
        chain's concat buffer holds y0, y1 only: stride 2c in the same
        allocation)."""
        h, w, c, f32, off = self.bufs[buf]
        c = cs or c
        n = self.B * h * w * c
        if f32:
            return self.ws[off:off + 4 * n].view(np.float32).reshape(self.B, h, w, c)
        return bf16_to_f32(self.ws[off:off + 2 * n].view(np.uint16)).reshape(self.B, h, w, c)


def _setup(cuda, H, W, B, variant=0):
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    flat = weights.synthetic_weights(variant, seed=1)
    eng = YoloEngine(variant, flat, B, (H, W), device=cuda)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=30 + b)), 3)
                   for b in range(B)])
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda))
    raw = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb, raw)
    specs, _ = yolo_ref.conv_specs(variant)
    params, off = {}, 0
    for n, ci, co, k, s, act in specs:
        nw = co * ci * k * k
        params[n] = (flat[off:off + nw].reshape(co, ci, k, k), flat[off + nw:off + nw + co])
        off += nw + co
    return eng, Introspect(eng, B), specs, params, lb.cpu().numpy(), raw.cpu().numpy()


@pytest.mark.parametrize("H,W,B,variant", [(640, 640, 1, 0), (1080, 1920, 2, 0),
                                            (640, 640, 1, 2)])  # 2 = YOLOv8m (config 5)
def test_every_conv_layerwise(cuda, H, W, B, variant):
    eng, ins, specs, params, lb, raw = _setup(cuda, H, W, B, variant)
    assert len(ins.recs) == len(specs) - 1  # all but model.0 go through conv_mfma
    worst = []
    for r in ins.recs:
        (ci_, inb, incs, inco, Hin, Win, Ho, Wo, o0, o0cs, o0co, up0, o1, o1cs, o1co, up1,
         rb, rcs, rco, in_up, in2b, in2cs, in2co, split) = r.tolist()
        name, cin, cout, k, s, act = specs[ci_]
        w, b = params[name]
        if in2b >= 0:  # virtual concat: [upsampled] view 1 channels, then view 2's
            x1 = ins.view(inb)[..., inco:inco + split]
            if in_up:
                x1 = x1.repeat(2, axis=1).repeat(2, axis=2)
            x = np.concatenate([x1, ins.view(in2b)[..., in2co:in2co + cin - split]], -1)
        else:
            x = ins.view(inb)[..., inco:inco + cin]
        xt = torch.from_numpy(np.ascontiguousarray(x.transpose(0, 3, 1, 2))).double()
        wt = torch.from_numpy(round_bf16(w)).double()
        y = F.conv2d(xt, wt, torch.from_numpy(b).double(), stride=s, padding=k // 2)
        if act:
            y = F.silu(y)
        y = y.numpy().transpose(0, 2, 3, 1)
        if rb >= 0:
            y = y + ins.view(rb)[..., rco:rco + cout]
        got = ins.view(o0)[..., o0co:o0co + cout]
        if up0:
            got = got[:, ::2, ::2]
        rms = float(np.sqrt(np.mean(y ** 2))) + 1e-12
        d = np.abs(got.astype(np.float64) - y)
        if ins.bufs[o0][3]:  # f32 head logits
            assert (d <= 1e-4 * rms + 1e-5 * np.abs(y)).all(), f"{name}: f32 max {d.max()}"
            continue
        tol1 = ulp_bf16(y) * 1.01 + 1e-3 * rms
        frac = float((d > tol1).mean())
        worst.append((frac, name))
        assert frac < 1e-4, f"{name}: {frac:.2e} of elements beyond 1 ulp"
        assert (d <= 2 * ulp_bf16(y) + 1e-2 * rms).all(), f"{name}: max dev {d.max()}"
        if o1 >= 0:  # second destination (concat slice or upsampled copy)
            g1 = ins.view(o1)[..., o1co:o1co + cout]
            for dy in ((0, 1) if up1 else (0,)):
                for dx in ((0, 1) if up1 else (0,)):
                    part = g1[:, dy::2, dx::2] if up1 else g1
                    np.testing.assert_array_equal(part, got, err_msg=name)
    print("worst layers:", sorted(worst)[-3:])


def test_first_conv_sppf_and_decode(cuda):
    H, W, B = 1080, 1920, 1
    eng, ins, specs, params, lb, raw = _setup(cuda, H, W, B)
    # model.0: 3->16 k3 s2 from the u8 letterbox, f32 math
    w, b = params["model.0"]
    x = torch.from_numpy(lb[..., ::-1].transpose(0, 3, 1, 2).copy()).double() / 255
    y = F.silu(F.conv2d(x, torch.from_numpy(w).double(), torch.from_numpy(b).double(), stride=2,
                        padding=1)).numpy().transpose(0, 2, 3, 1)
    got = ins.view(0)
    d = np.abs(got - y)
    assert (d <= ulp_bf16(y) * 1.01 + 1e-6).mean() > 0.9999 and (d <= 2 * ulp_bf16(y) + 1e-5).all()
    # SPPF: channels [c,2c,3c,4c) are 5/9/13 max pools of [0,c) (exact)
    sp = [i for i, bb in enumerate(ins.bufs) if bb[2] == 4 * (256 // 2) and bb[0] == 384 // 32]
    assert sp, "SPPF buffer not found"
    s = ins.view(sp[0])
    c = s.shape[-1] // 4
    t = torch.from_numpy(np.ascontiguousarray(s[..., :c].transpose(0, 3, 1, 2)))
    p1 = F.max_pool2d(t, 5, 1, 2)
    p2 = F.max_pool2d(p1, 5, 1, 2)
    p3 = F.max_pool2d(p2, 5, 1, 2)
    for j, p in enumerate((p1, p2, p3)):
        np.testing.assert_array_equal(s[..., (j + 1) * c:(j + 2) * c], p.numpy().transpose(0, 2, 3, 1))
    # decode from the GPU's own head logits
    # (the f32 logit maps: 4 * reg_max + nc channels; the chained head's
    # small f32 maps -- DFL distances, (score, class) -- are not logits)
    heads = [i for i, bb in enumerate(ins.bufs) if bb[3] == 1 and bb[2] == 4 * 16 + 80]
    assert len(heads) == 3
    outs, anc, st = [], [], []
    for lvl, hb in enumerate(heads):
        v = ins.view(hb)  # (B, h, w, 144)
        h, w = v.shape[1:3]
        outs.append(v.reshape(B, h * w, -1).transpose(0, 2, 1))
        sy, sx = np.meshgrid(np.arange(h) + 0.5, np.arange(w) + 0.5, indexing="ij")
        anc.append(np.stack([sx.ravel(), sy.ravel()]))
        st.append(np.full(h * w, 8.0 * 2 ** lvl))
    y = np.concatenate(outs, 2).astype(np.float64)
    A = y.shape[2]
    box = y[:, :64].reshape(B, 4, 16, A)
    e = np.exp(box - box.max(2, keepdims=True))
    dist = (e / e.sum(2, keepdims=True) * np.arange(16).reshape(1, 1, 16, 1)).sum(2)
    an = np.concatenate(anc, 1)[None]
    s_ = np.concatenate(st)[None]
    x1y1, x2y2 = an - dist[:, :2], an + dist[:, 2:]
    xywh = np.concatenate([(x1y1 + x2y2) / 2, x2y2 - x1y1], 1) * s_[:, None]
    np.testing.assert_allclose(raw[:, :4], xywh, rtol=0, atol=2e-3)
    np.testing.assert_allclose(raw[:, 4:], 1 / (1 + np.exp(-y[:, 64:])), rtol=0, atol=1e-6)
    # candidates: every anchor with best score > conf, none else
    n = int(eng.seg_n.view(-1)[:eng.nseg].sum())  # image 0's segments
    expect = int((raw[0, 4:].max(0) > 0.25).sum())
    assert n == expect


def test_autotuned_configs_are_bit_identical(cuda):
    """rv_yolo_autotune times every valid kernel configuration of every conv
    launch (tile shape, chunk group, resident weights) and checks each
    configuration's output buffers against the default's: all accumulate in
    the same k order, so they must agree bit for bit.  The tuned forward must
    then reproduce the default forward's raw prediction exactly."""
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    H, W, B = 1080, 1920, 2
    eng = YoloEngine(0, weights.synthetic_weights(0, seed=2), B, (H, W), device=cuda)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=50 + b)), 3) for b in range(B)])
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda))
    raw0 = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb, raw0)
    assert eng.autotune(lb, reps=1, verify=True) == 0
    cfgs = eng.tuned_configs()
    assert len(cfgs) > 0 and all(c[0] >= 0 for c in cfgs)
    raw1 = torch.empty_like(raw0)
    eng.forward_raw(lb, raw1)
    np.testing.assert_array_equal(raw1.cpu().numpy(), raw0.cpu().numpy())
    eng.close()


def test_fused_stem_matches_unfused(cuda):
    """conv0 + model.1 (+ model.2.cv1 from the registers) fused (X0 kept in
    LDS, model.1 on tap pairs) against the unfused launches: same X0 values,
    model.1 accumulated in another k order, so X1 agrees to 1 bf16 ulp (fewer
    than 1e-4 of the elements beyond); model.2.cv1 computed by the stem from
    ITS X1 is bit-identical to the unfused 1x1 kernel run on that X1."""
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    H, W, B = 1080, 1920, 2
    eng = YoloEngine(0, weights.synthetic_weights(0, seed=3), B, (H, W), device=cuda)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=70 + b)), 3) for b in range(B)])
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda))
    eng.set_stem_x1(True)
    eng.forward_raw(lb)  # no raw output: fused stem (+ X1 for this test)
    ins = Introspect(eng, B)
    x1_fused = ins.view(1).copy()
    c2 = [i for i, bb in enumerate(ins.bufs) if bb[2] == 48 and bb[0] == 96][0]
    cv1_fused = ins.view(c2, cs=32).copy()  # fused model.2: [y0 | y1] only
    raw = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb, raw)  # raw output requested: conv0 + model.1 separately
    ins2 = Introspect(eng, B)
    x1 = ins2.view(1)
    assert x1.shape == (B, 96, 160, 32)
    rms = float(np.sqrt(np.mean(x1.astype(np.float64) ** 2))) + 1e-12
    d = np.abs(x1_fused.astype(np.float64) - x1)
    assert float((d > ulp_bf16(x1) * 1.01 + 1e-3 * rms).mean()) < 1e-4
    assert (d <= 2 * ulp_bf16(x1) + 1e-2 * rms).all()
    # cv1 of the fused stem vs a float64 recomputation from the fused X1
    specs, params = yolo_ref.conv_specs(0)[0], {}
    flat = weights.synthetic_weights(0, seed=3)
    off = 0
    for n, ci, co, k, s, act in specs:
        nw = co * ci * k * k
        params[n] = (flat[off:off + nw].reshape(co, ci), flat[off + nw:off + nw + co]) if k == 1 \
            else None
        off += nw + co
    w, b = params["model.2.cv1"]
    y = x1_fused.astype(np.float64) @ round_bf16(w).astype(np.float64).T + b
    y = y / (1 + np.exp(-y))
    rms = float(np.sqrt(np.mean(y ** 2))) + 1e-12
    d = np.abs(cv1_fused - y)
    assert float((d > ulp_bf16(y) * 1.01 + 1e-3 * rms).mean()) < 1e-4
    assert (d <= 2 * ulp_bf16(y) + 1e-2 * rms).all()
    eng.close()


def test_stem_cv1_bit_identical_to_unfused_1x1(cuda):
    """The stem's fused model.2.cv1 against the unfused 1x1 kernels on the
    same X1 bits: run the production forward with X1 written, then the
    unfused model.2.cv1 kernel is reproduced by the raw forward's layer on
    that X1 -- the raw (unfused) forward recomputes X1 itself, so instead the
    C2 slice of the fused forward is compared with the raw forward's C2
    slice wherever the two X1 maps agree bit for bit over the 1x1 support
    (the pixel itself)."""
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    H, W, B = 1080, 1920, 2
    eng = YoloEngine(0, weights.synthetic_weights(0, seed=3), B, (H, W), device=cuda)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=70 + b)), 3) for b in range(B)])
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda))
    eng.set_stem_x1(True)
    eng.forward_raw(lb)
    ins = Introspect(eng, B)
    x1_f = ins.raw_u16(1).copy()
    c2 = [i for i, bb in enumerate(ins.bufs) if bb[2] == 48 and bb[0] == 96][0]
    cv1_f = ins.raw_u16(c2, cs=32).copy()  # fused model.2: [y0 | y1] only
    raw = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb, raw)
    ins2 = Introspect(eng, B)
    x1_u = ins2.raw_u16(1)
    cv1_u = ins2.raw_u16(c2)[..., :32]
    same = (x1_f == x1_u).all(-1)
    assert same.mean() > 0.9
    np.testing.assert_array_equal(cv1_f[same], cv1_u[same])
    eng.close()


@pytest.mark.parametrize("cfg", [None, (4, 2, 1, 1, 1, 2), (4, 2, 1, 1, 1, 0), (2, 2, 1, 1, 1, 0),
                                 (4, 1, 1, 0, 1, 2), (2, 4, 1, 1, 1, 0)])
def test_residual_conv_exact_allocation(cuda, cfg):
    """A 3x3 bf16 conv + SiLU + residual (the bottleneck form) through
    rv_conv_bf16 with the residual in its own exactly-sized allocation and
    Ho, Wo not multiples of any tile height: the deferred-store epilogue
    (tiles up to 10 fragments) must not read the residual past its end for
    the bottom tile row's invalid pixels, and the output equals
    a float64 recomputation to 1 bf16 ulp."""
    from rvs_amd import _lib
    B, H, W, C = 2, 37, 45, 64
    g = torch.Generator().manual_seed(11)
    x = (torch.randn((B, H, W, C), generator=g) * 0.5).to(torch.bfloat16)
    wt = (torch.randn((C, C, 3, 3), generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(C, generator=g) * 0.1
    res = (torch.randn((B, H, W, C), generator=g) * 0.5).to(torch.bfloat16)
    wp = torch.zeros((C, 9, 32 * ((C + 31) // 32)), dtype=torch.bfloat16)
    wp[:, :, :C] = wt.permute(0, 2, 3, 1).reshape(C, 9, C)
    xd, wd, bd, rd = x.to(cuda), wp.to(cuda), b.to(cuda), res.to(cuda).clone()
    out = torch.full((B, H, W, C), float("nan"), dtype=torch.bfloat16, device=cuda)
    cfg_arr = _lib.int_array(cfg) if cfg is not None else None
    st = _lib.load().rv_conv_bf16(_lib.ptr(xd), B, H, W, C, C, _lib.ptr(wd), _lib.ptr(bd), C, 3, 1,
                                  _lib.ptr(out), C, _lib.ptr(rd), C, 1, cfg_arr, _lib.stream_ptr())
    if cfg is not None and st != 0:
        pytest.skip(f"configuration {cfg} not valid for this layer")
    assert st == 0
    torch.cuda.synchronize()
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), wt.double(), b.double(), padding=1)
    ref = ref * torch.sigmoid(ref)
    ref = (ref.permute(0, 2, 3, 1) + res.double()).numpy()
    got = out.float().cpu().numpy().astype(np.float64)
    assert np.isfinite(got).all()
    rms = float(np.sqrt(np.mean(ref ** 2)))
    d = np.abs(got - ref)
    assert (d <= 2 * ulp_bf16(ref) + 1e-3 * rms).all()


@pytest.mark.parametrize("H,W,B,variant", [(1080, 1920, 3, 0), (640, 640, 1, 0), (360, 640, 2, 0)])
def test_fused_c2f_is_bit_identical(cuda, H, W, B, variant):
    """The fused C2f chains (c2f.hip: model.2 / model.4 / model.15 bottlenecks
    + cv2 in one launch each, intermediates in LDS) against one launch per
    conv, on the production kernel sequence: every output map of the blocks,
    the raw prediction and the NMS candidates are bit-identical (same MFMA
    k-order and epilogue; the width-16 chain with its per-tap k-steps,
    RV_YOLO_OPT_C2F_TAP_PAIRS = 0)."""
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    eng = YoloEngine(variant, weights.synthetic_weights(variant, seed=5), B, (H, W), device=cuda)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=90 + b)), 3) for b in range(B)])
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda))
    eng.set_raw_fused(True)
    eng.set_c2f_tap_pairs(False)
    outs = []
    for fuse in (False, True):
        eng.set_fuse_c2f(2 if fuse else 0)  # every fusable chain (the default fuses C = 16 only)
        raw = torch.full((B, 84, eng.A), float("nan"), dtype=torch.float32, device=cuda)
        eng.forward_raw(lb, raw, slot=int(fuse))
        torch.cuda.synchronize()
        ins = Introspect(eng, B)
        # outputs of the fused blocks: X2 (model.2), the CAT14 slice of model.4,
        # X15 (model.15) -- located through the trace of the last forward
        specs, _ = yolo_ref.conv_specs(variant)
        maps = {}
        for rec in ins.recs:
            name, cout = specs[rec[0]][0], specs[rec[0]][2]
            if name in ("model.2.cv2", "model.4.cv2", "model.15.cv2"):
                maps[name] = ins.view(rec[8])[..., rec[10]:rec[10] + cout].copy()
        seg = eng.seg_n[int(fuse)].cpu().numpy().copy()
        outs.append((raw.cpu().numpy(), maps, seg))
    (r0, m0, s0), (r1, m1, s1) = outs
    assert set(m0) == {"model.2.cv2", "model.4.cv2", "model.15.cv2"} == set(m1)
    for k in m0:
        np.testing.assert_array_equal(m1[k], m0[k], err_msg=k)
    np.testing.assert_array_equal(r1, r0)
    np.testing.assert_array_equal(s1, s0)
    eng.close()


@pytest.mark.parametrize("H,W,B", [(1080, 1920, 3), (640, 640, 1), (360, 640, 2)])
def test_c2f_tap_pairs_within_one_ulp(cuda, H, W, B):
    """The production width-16 C2f chain (model.2: its 3x3 convs on tap
    pairs, two taps' 16 channels per 32-deep MFMA k-step) against the
    per-tap k order (bit-identical to the unfused launches): the block's
    output X2 agrees to 1 bf16 ulp (fewer than 1e-3 of the elements beyond,
    none beyond 2 ulp + 1e-2 rms -- the stem's model.1 bar), and the
    forward's candidates per image stay within 1 % of each other.  (On
    MI355X the two k orders have agreed bit for bit on every input measured:
    the zero upper k-half of a per-tap step adds nothing, so both add the
    same products in the same k order; the bar stays at 1 ulp.)"""
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    eng = YoloEngine(0, weights.synthetic_weights(0, seed=5), B, (H, W), device=cuda)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=95 + b)), 3) for b in range(B)])
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda))
    eng.set_raw_fused(True)
    outs = []
    for pairs in (False, True):
        eng.set_c2f_tap_pairs(pairs)
        raw = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
        eng.forward_raw(lb, raw, slot=int(pairs))
        torch.cuda.synchronize()
        ins = Introspect(eng, B)
        specs, _ = yolo_ref.conv_specs(0)
        x2 = None
        for rec in ins.recs:
            if specs[rec[0]][0] == "model.2.cv2":
                x2 = ins.view(rec[8])[..., rec[10]:rec[10] + specs[rec[0]][2]].copy()
        nseg = eng.nseg
        seg = eng.seg_n[int(pairs)].view(-1)[:B * nseg].view(B, nseg).cpu().numpy().copy()
        outs.append((x2, raw.cpu().numpy(), seg))
    (x0, r0, s0), (x1, r1, s1) = outs
    assert x0 is not None and x0.shape == x1.shape
    rms = float(np.sqrt(np.mean(x0.astype(np.float64) ** 2))) + 1e-12
    d = np.abs(x1.astype(np.float64) - x0)
    assert float((d > ulp_bf16(x0) * 1.01 + 1e-3 * rms).mean()) < 1e-3
    assert (d <= 2 * ulp_bf16(x0) + 1e-2 * rms).all()
    assert np.isfinite(r1).all()
    n0, n1 = s0.sum(axis=-1), s1.sum(axis=-1)
    assert (np.abs(n1 - n0) <= 0.01 * np.maximum(n0, 100)).all()
    eng.close()


@pytest.mark.parametrize("H,W,B", [(1080, 1920, 3), (640, 640, 2), (360, 640, 1)])
def test_chained_cv1_is_bit_identical(cuda, H, W, B):
    """model.3 with model.4.cv1 chained in the same launch (the 1x1 runs on
    model.3's output tile in LDS; conv_patch_kernel CH form) against the two
    launches, on the production kernel sequence, default and every autotuned
    configuration: cv1's output (the y0 | y1 slice of model.4's concat
    buffer), the raw prediction and the NMS candidates are bit-identical."""
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    eng = YoloEngine(0, weights.synthetic_weights(0, seed=7), B, (H, W), device=cuda)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=40 + b)), 3) for b in range(B)])
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda))
    eng.set_raw_fused(True)
    specs, _ = yolo_ref.conv_specs(0)

    def run(chain, slot):
        eng.set_fuse_cv1(chain)
        raw = torch.full((B, 84, eng.A), float("nan"), dtype=torch.float32, device=cuda)
        eng.forward_raw(lb, raw, slot=slot)
        torch.cuda.synchronize()
        ins = Introspect(eng, B)
        cv1 = None
        for rec in ins.recs:
            if specs[rec[0]][0] == "model.4.cv1":
                cv1 = ins.view(rec[8])[..., rec[10]:rec[10] + specs[rec[0]][2]].copy()
        assert cv1 is not None
        return raw.cpu().numpy(), cv1, eng.seg_n[slot].cpu().numpy().copy()

    r0, c0, s0 = run(False, 0)
    for tuned in (False, True):
        if tuned:
            eng.autotune(lb, reps=1)
        r1, c1, s1 = run(True, 1)
        np.testing.assert_array_equal(c1, c0)
        np.testing.assert_array_equal(r1, r0)
        np.testing.assert_array_equal(s1, s0)
    # the chained launch is one record of the production launch list
    assert sum(1 for c in eng.tuned_configs() if c) >= 1
    eng.close()


@pytest.mark.parametrize("H,W,B", [(1080, 1920, 4), (640, 640, 2), (360, 640, 3)])
def test_chained_head_matches_decode(cuda, H, W, B):
    """The chained Detect head (each branch's last 1x1 conv in its 3x3
    conv's launch: box + DFL, class + sigmoid / first maximum; then the
    combine kernel) against the decode kernel on the same forward: every
    segment's candidate count and rows, and the NMS output, bit-identical
    -- default and autotuned conv configurations."""
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    eng = YoloEngine(0, weights.synthetic_weights(0, seed=11), B, (H, W), device=cuda)
    fr = np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=60 + b)), 3) for b in range(B)])
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda))

    def run(chain, slot):
        eng.set_head_chain(chain)
        eng.seg_n[slot].fill_(-7)
        eng.forward_raw(lb, slot=slot)
        dets, n = eng.nms(B, slot)
        torch.cuda.synchronize()
        nseg = eng.nseg
        seg = eng.seg_n[slot].view(-1)[:B * nseg].view(B, nseg).cpu().numpy().copy()
        cand = eng.cand[slot][:B].cpu().numpy().view(np.uint32).reshape(B, eng.cap, -1)
        rows = [cand[b, 64 * j:64 * j + seg[b, j]].copy() for b in range(B) for j in range(nseg)]
        return seg, rows, dets.cpu().numpy().copy(), n.cpu().numpy().copy()

    s0, r0, d0, n0 = run(False, 0)
    assert s0.min() >= 0 and s0.sum() > 0
    for tuned in (False, True):
        if tuned:
            eng.autotune(lb, reps=1)
        s1, r1, d1, n1 = run(True, 1)
        np.testing.assert_array_equal(s1, s0)
        for a, b in zip(r1, r0):
            np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(n1, n0)
        np.testing.assert_array_equal(d1.view(np.uint32), d0.view(np.uint32))
    eng.close()
