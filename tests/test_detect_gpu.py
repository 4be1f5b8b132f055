"""Detector HIP path vs the CPU oracle (oracle/yolo_ref.py).

Tolerances (stated here, see DESIGN.md "Parity"):
  * NMS + scale_boxes + class filter on the SAME raw prediction: bit-exact
    (boxes, scores, classes and order).
  * Every conv kernel is checked layer by layer (test_yolo_layers_gpu.py:
    within 1 bf16 ulp of a float64 recomputation from the GPU's own inputs).
  * Whole-network comparisons are statistical: a bf16 rounding that flips
    because of a different f32 accumulation order moves later layers.  The
    synthetic weights are calibrated into the ordered regime
    (tests/golden/make_yolo_scales.py; round 1's were chaotic: input noise
    1e-4 moved boxes 2.8 px at p99, now 0.5 px on candidate anchors).
    Measured and asserted here:
      - vs the torch-CPU restatement at the same storage precision
        (quant=True: bf16 weights/activations, f32 accumulate): class-score
        |d| <= 0.005 at the 99.9th percentile, box xywh |d| <= 1 px + 1 % for
        >= 99.9 % of anchors;
      - vs the pure fp32 restatement (the reference's precision):
        class-score |d| <= 0.01 at p99.9, box |d| <= 2 px + 2 % for >= 99.9 %;
      - end to end (letterbox -> forward -> NMS -> class filter): >= 95 % of
        the quantised oracle's detections matched by a GPU detection of the
        same class with IoU >= 0.9 and vice versa (>= 85 % vs fp32).
    Ultralytics itself is absent, so detector parity against real
    Ultralytics (and real weights) is unpinned.
"""
import numpy as np
import pytest
import torch

from conftest import road_frame
from oracle import cpu, yolo_ref

pytestmark = pytest.mark.gpu


def _engine(H, W, B, cuda, variant=0, **kw):
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    flat = weights.synthetic_weights(variant, seed=0)
    return YoloEngine(variant, flat, B, (H, W), device=cuda, **kw), flat


def _frames(H, W, B, seed=0):
    return np.stack([cpu.median(cpu.clahe_ycrcb(road_frame(H, W, seed=seed + b)), 3)
                     for b in range(B)])


@pytest.mark.parametrize("H,W,B", [(640, 640, 1), (1080, 1920, 2)])
@pytest.mark.parametrize("quant", [True, False])
def test_forward_matches_oracle(cuda, H, W, B, quant):
    eng, flat = _engine(H, W, B, cuda)
    fr = _frames(H, W, B)
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda))
    raw = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb, raw, candidates=False)
    got = raw.cpu().numpy()
    ref = yolo_ref.YoloRef(0, flat, quant=quant).forward(
        yolo_ref.preprocess(lb.cpu().numpy())).numpy()
    assert got.shape == ref.shape
    ds = np.abs(got[:, 4:] - ref[:, 4:])
    db = np.abs(got[:, :4] - ref[:, :4])
    if quant:  # measured r02: score p99.9 0.0033, 99.99 % of boxes within 1 px + 1 %
        s_tol, b_abs, b_rel, b_frac = 0.005, 1.0, 0.01, 0.999
    else:  # measured r02: score p99.9 0.0061, box p99 2.4 px
        s_tol, b_abs, b_rel, b_frac = 0.01, 2.0, 0.02, 0.999
    frac_box = float((db <= b_abs + b_rel * np.abs(ref[:, :4])).mean())
    print(f"quant={quant} score |d| max {ds.max():.4f} p99.9 {np.percentile(ds, 99.9):.4f}; "
          f"box |d| max {db.max():.2f} px p99 {np.percentile(db, 99):.3f}, "
          f"within tol {frac_box:.5f}")
    assert np.percentile(ds, 99.9) <= s_tol
    assert frac_box >= b_frac


def test_nms_bit_exact_on_same_raw(cuda):
    H, W, B = 1080, 1920, 3
    eng, flat = _engine(H, W, B, cuda, classes_keep=[0, 2, 3, 5, 7])
    fr = _frames(H, W, B, seed=10)
    lb = eng.letterbox(torch.from_numpy(fr).to(cuda)).cpu().numpy()
    raw = yolo_ref.YoloRef(0, flat).forward(yolo_ref.preprocess(lb)).numpy()
    dets, n = eng.nms_from_raw(torch.from_numpy(raw).to(cuda))
    dets, n = dets.cpu().numpy(), n.cpu().numpy()
    ref = yolo_ref.postprocess(raw, (eng.in_h, eng.in_w), (H, W), classes_keep=[0, 2, 3, 5, 7])
    for b in range(B):
        np.testing.assert_array_equal(dets[b, :n[b]], ref[b])


def _raw_from_boxes(boxes, scores, cls, A, nc=80):
    raw = np.zeros((1, 4 + nc, A), np.float32)
    n = len(boxes)
    b = np.asarray(boxes, np.float32)
    raw[0, 0, :n] = (b[:, 0] + b[:, 2]) / 2
    raw[0, 1, :n] = (b[:, 1] + b[:, 3]) / 2
    raw[0, 2, :n] = b[:, 2] - b[:, 0]
    raw[0, 3, :n] = b[:, 3] - b[:, 1]
    raw[0, 4 + np.asarray(cls), np.arange(n)] = scores
    return raw


# "overflow": more candidates than the first NMS pass sorts in LDS (4096), so
# the image is redone by the overflow pass (keys in global memory);
# "maxnms": Ultralytics' max_nms cut (top max_nms by score) at a small max_nms
@pytest.mark.parametrize("case", ["ties", "dense", "empty", "many", "overflow", "maxdet", "classes",
                                  "maxnms"])
def test_nms_edge_cases(cuda, case):
    rng = np.random.default_rng(hash(case) % 2**32)
    A = 5040
    max_nms = 64 if case == "maxnms" else 30000
    eng, _ = _engine(1080, 1920, 1, cuda, max_det=100 if case != "maxdet" else 7,
                     classes_keep=[2, 7] if case == "classes" else (), max_nms=max_nms)
    if case == "empty":
        boxes, scores, cls = np.zeros((0, 4)), np.zeros(0), np.zeros(0, int)
    else:
        n = {"ties": 300, "dense": 400, "many": 4000, "overflow": 5000, "maxdet": 200,
             "classes": 500, "maxnms": 400}[case]
        xy = rng.uniform(0, 600, (n, 2))
        wh = rng.uniform(10, 120, (n, 2)) if case != "dense" else rng.uniform(200, 260, (n, 2))
        boxes = np.concatenate([xy, xy + wh], 1)
        scores = rng.uniform(0.26, 1.0, n)
        cls = rng.integers(0, 80 if case != "dense" else 3, n)
        if case == "ties":
            scores = np.round(scores * 8) / 8  # heavy score ties
            scores[scores <= 0.25] = 0.375
            boxes[::7] = boxes[0]
            cls[::7] = cls[0]
    raw = _raw_from_boxes(boxes, scores, cls, A)
    dets, n_ = eng.nms_from_raw(torch.from_numpy(raw).to(cuda))
    ref = yolo_ref.postprocess(raw, (eng.in_h, eng.in_w), (1080, 1920), max_det=eng.max_det,
                               max_nms=max_nms, classes_keep=[2, 7] if case == "classes" else ())
    np.testing.assert_array_equal(dets[0, :int(n_[0])].cpu().numpy(), ref[0])
    if case == "maxnms":
        assert int(n_[0]) > 0


@pytest.mark.parametrize("n", [20000, 33500])
def test_nms_config5_candidates(cuda, n):
    """Config 5 geometry (1280 x 1280, A = 33600 anchors): more candidates
    than 16384, and (n = 33500) more than max_nms = 30000.  Every candidate
    is sorted; only the top 30000 by score enter the greedy pass (Ultralytics
    max_nms).  Boxes sit in tight same-class clusters (NMS keeps about one per
    cluster and class); the 3500 lowest-score boxes form clusters of their own,
    so they reach the output exactly when they survive the max_nms cut."""
    rng = np.random.default_rng(n)
    eng, _ = _engine(1280, 1280, 1, cuda, imgsz=1280, max_det=1024)
    A = eng.A
    assert A == 33600
    n_low = 3500

    def clusters(m, nclu, lo, hi):
        ctr = rng.uniform(lo, hi, (nclu, 2))
        k = rng.integers(0, nclu, m)
        xy = ctr[k] + rng.normal(0, 1.0, (m, 2))
        return np.concatenate([xy, xy + 60.0 + rng.normal(0, 1.0, (m, 2))], 1), k % 4

    b_lo, c_lo = clusters(n_low, 20, 1000, 1180)
    b_hi, c_hi = clusters(n - n_low, 64, 0, 900)
    boxes = np.concatenate([b_lo, b_hi])
    cls = np.concatenate([c_lo, c_hi])
    scores = np.concatenate([np.sort(rng.uniform(0.26, 0.4, n_low)),
                             rng.uniform(0.5, 1.0, n - n_low)])
    raw = _raw_from_boxes(boxes, scores, cls, A)
    dets, n_ = eng.nms_from_raw(torch.from_numpy(raw).to(cuda))
    ref = yolo_ref.postprocess(raw, (eng.in_h, eng.in_w), (1280, 1280), max_det=1024)
    got = dets[0, :int(n_[0])].cpu().numpy()
    np.testing.assert_array_equal(got, ref[0])
    assert int(eng.cand_n[0]) == n
    low_kept = int((got[:, 4] < 0.45).sum())
    print(f"n={n}: kept {len(got)}, low-score kept {low_kept}")
    assert len(got) < 1024
    assert (low_kept == 0) if n > 30000 else (low_kept > 0)


def _iou(a, b):
    x1, y1 = max(a[0], b[0]), max(a[1], b[1])
    x2, y2 = min(a[2], b[2]), min(a[3], b[3])
    inter = max(0, x2 - x1) * max(0, y2 - y1)
    u = (a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter
    return inter / u if u > 0 else 0


@pytest.mark.parametrize("H,W,B", [(1080, 1920, 4), (640, 640, 3)])
def test_register_head_candidates_equal_lds_path(cuda, H, W, B):
    """Without a raw output the YOLOv8n head decode keeps the class scores in
    registers (detect_decode_kernel<..., NCT = 80>, blocks walking 4 anchor
    tiles); with one it takes the LDS path that also writes raw.  Their
    candidate segments are bit-identical: counts, boxes, scores, classes,
    anchors and order."""
    eng, _ = _engine(H, W, B, cuda)
    lb = eng.letterbox(torch.from_numpy(_frames(H, W, B, seed=7)).to(cuda))
    out = []
    for with_raw in (False, True):
        eng.cand[0].zero_()
        eng.seg_n[0].zero_()
        raw = torch.empty((B, 4 + eng.nc, eng.A), dtype=torch.float32,
                          device=cuda) if with_raw else None
        eng.forward_raw(lb, raw=raw)
        torch.cuda.synchronize()
        out.append((eng.seg_n[0, :B].cpu().numpy(), eng.cand[0, :B].cpu().numpy().view(np.int32)))
    (n0, c0), (n1, c1) = out
    assert np.array_equal(n0, n1) and n0.sum() > 0
    for b in range(B):
        for j in np.nonzero(n0[b])[0]:
            k = int(n0[b, j])
            assert np.array_equal(c0[b, 64 * j:64 * j + k], c1[b, 64 * j:64 * j + k]), (b, j)


def _match_frac(a, b, min_score=0.27):
    """Fraction of the rows of `a` with score >= min_score matched by a row of
    `b` with the same class and IoU >= 0.9 (per image lists of (n, 6) rows).
    Rows within 0.02 of conf = 0.25 are left out: any change of the last
    bits decides whether such a candidate exists at all."""
    tot = hit = 0
    for x, y in zip(a, b):
        for r in x:
            if r[4] < min_score:
                continue
            tot += 1
            hit += any(int(g[5]) == int(r[5]) and _iou(g, r) >= 0.9 for g in y)
    return hit, tot


@pytest.mark.parametrize("H,W", [(1080, 1920), (640, 640)])
def test_end_to_end_detections(cuda, H, W):
    """letterbox -> forward -> NMS -> class filter on the GPU vs the oracle's
    detections (the reference's default classes_keep [0, 2, 3, 5, 7]).
    Against YoloRef(quant=True) -- the same storage precision (bf16 weights
    and activations, f32 accumulation), so the two differ only in
    accumulation order and the hardware exp / reciprocal: >= 95 % of the
    detections match (same class, IoU >= 0.9) in both directions.  The
    oracle's own floor under a 1e-7 relative change of every conv output
    before its bf16 rounding is ~96-98 % (tools/calib_search.py; NMS picks
    between near-tied overlapping candidates).  Against the fp32 restatement
    (the reference's precision): >= 85 % (bf16 storage itself, measured
    offline at ~90 %)."""
    B = 4
    keep = [0, 2, 3, 5, 7]
    eng, flat = _engine(H, W, B, cuda, classes_keep=keep)
    fr = _frames(H, W, B, seed=20)
    dets, n = eng.run(torch.from_numpy(fr).to(cuda))
    dets, n = dets.cpu().numpy(), n.cpu().numpy()
    got = [dets[b, :n[b]] for b in range(B)]
    lb = yolo_ref.preprocess(eng.letterbox(torch.from_numpy(fr).to(cuda)).cpu().numpy())
    out = {}
    for quant in (True, False):
        raw = yolo_ref.YoloRef(0, flat, quant=quant).forward(lb).numpy()
        ref = yolo_ref.postprocess(raw, (eng.in_h, eng.in_w), (H, W), classes_keep=keep)
        out[quant] = (_match_frac(ref, got), _match_frac(got, ref))
        print(f"quant={quant}: oracle dets matched by GPU {out[quant][0]}, "
              f"GPU dets matched by oracle {out[quant][1]}; all rows: {_match_frac(ref, got, 0)}")
    (h1, t1), (h2, t2) = out[True]
    assert t1 > 0 and h1 >= 0.95 * t1 and h2 >= 0.95 * t2
    (h1, t1), (h2, t2) = out[False]
    assert h1 >= 0.85 * t1 and h2 >= 0.85 * t2


def test_detector_api_returns_detections(cuda):
    from rvs_amd.detect import Detection, build_detector
    det = build_detector({"backend": "ultralytics", "model": "yolov8n.pt", "conf_thres": 0.25,
                          "iou_thres": 0.7, "max_det": 100, "classes_keep": [0, 2, 3, 5, 7]})
    img = road_frame(480, 640, seed=3)
    out = det.infer(img)
    assert isinstance(out, list) and all(isinstance(d, Detection) for d in out)
    for d in out:
        assert d.cls_id in (0, 2, 3, 5, 7) and d.track_id is None
        assert 0 <= d.x1 <= d.x2 <= 640 and 0 <= d.y1 <= d.y2 <= 480
    det.close()
