"""BASELINE config 5: YOLOv8m at 1280x1280, batch 16, on fog/rain-augmented
frames made on the device (rv_fog_rain_u8), in both plans: the fp8 MFMA
plan the config names (test_v8m_1280_fog_batch16_fp8) and the bf16 plan.

bf16 plan checks:
  * the fog generator feeds the detector directly (device-resident batch);
  * batch invariance: frame b of the batch-16 forward is bit-identical to the
    same frame run alone (every kernel's per-pixel reduction order is fixed);
  * one frame against the torch-CPU restatement at the HIP path's storage
    precision (oracle/yolo_ref.py quant=True).  Every YOLOv8m conv is within
    1 bf16 ulp of a float64 recomputation (test_yolo_layers_gpu.py, variant
    2), so the remaining whole-network gap is bf16 rounding flips carried
    through 83 convs of synthetic weights (test_detect_gpu.py).  Measured on
    MI355X (r02, ordered-regime weights): class-score |d| 0.0058 at p99.9,
    box xywh within 1 px + 1 % for 99.97 % of anchors.  Asserted:
    p99.9 <= 0.02 and >= 99.5 %;
  * NMS on the GPU's raw prediction is bit-exact against the restated NMS.
Layer-by-layer YOLOv8m parity is in test_yolo_layers_gpu.py (variant 2).
"""
import numpy as np
import pytest
import torch

from conftest import road_frame
from oracle import yolo_ref

pytestmark = pytest.mark.gpu


def test_v8m_1280_fog_batch16(cuda):
    from rvs_amd.augment import FogSynthesizer
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    H = W = 1280
    B = 16
    clean = torch.from_numpy(np.stack([road_frame(H, W, seed=70 + b) for b in range(4)]))
    clean = clean.to(cuda).repeat(4, 1, 1, 1)
    syn = FogSynthesizer(level="medium", seed=5, rain_p=0.002, device=cuda, filters=False)
    frames = syn.synthesize_batch(clean)
    assert not torch.equal(frames[0], frames[4])  # one draw per frame
    flat = weights.synthetic_weights(2, seed=0)
    eng = YoloEngine(2, flat, B, (H, W), imgsz=1280, device=cuda)
    assert (eng.in_h, eng.in_w) == (1280, 1280) and eng.A == 33600
    lb = eng.letterbox(frames)
    raw = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb, raw, candidates=False)
    one = torch.empty((1, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb[13:14].clone(), one, candidates=False)
    torch.cuda.synchronize()
    assert torch.equal(raw[13], one[0]), "batch-16 frame differs from the same frame alone"

    got = raw[:1].cpu().numpy()
    ref = yolo_ref.YoloRef(2, flat, quant=True).forward(
        yolo_ref.preprocess(lb[:1].cpu().numpy())).numpy()
    ds = np.abs(got[:, 4:] - ref[:, 4:])
    db = np.abs(got[:, :4] - ref[:, :4])
    frac_box = float((db <= 1.0 + 0.01 * np.abs(ref[:, :4])).mean())
    print(f"v8m 1280: score |d| p99.9 {np.percentile(ds, 99.9):.4f} max {ds.max():.4f}; "
          f"box within tol {frac_box:.5f}")
    # measured r02 (ordered-regime synthetic weights): score p99.9 0.0058,
    # 99.97 % of box coordinates within 1 px + 1 %
    assert np.percentile(ds, 99.9) <= 0.02
    assert frac_box >= 0.995

    dets, n = eng.nms_from_raw(raw)
    dets, n = dets.cpu().numpy(), n.cpu().numpy()
    ref_d = yolo_ref.postprocess(raw.cpu().numpy(), (H, W), (H, W))
    for b in range(B):
        np.testing.assert_array_equal(dets[b, :n[b]], ref_d[b].astype(np.float32).reshape(-1, 6))
    assert n.sum() > 0
    eng.close()


def test_v8m_1280_fog_batch16_fp8(cuda):
    """configs[4] as named: YOLOv8m, 1280x1280, batch 16, fp8 (OCP e4m3)
    MFMA plan on device-made fog/rain frames, activation scales calibrated on
    the batch.  Frame 0 and frame 9 against YoloRef(quant="fp8") with the
    GPU's scales: >= 90 % of the oracle's detections matched by a GPU
    detection of the same class at IoU >= 0.9 and vice versa (the oracle's
    own floor under accumulation-order perturbations is 95-97.5 %,
    tests/test_fp8_gpu.py); >= 80 % of the GPU's detections have a
    same-class fp32-oracle detection at IoU >= 0.5; batch invariance of the
    fp8 plan; NMS exact on the GPU's raw prediction."""
    from rvs_amd.augment import FogSynthesizer
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    from test_fp8_gpu import _match
    H = W = 1280
    B, keep = 16, [0, 2, 3, 5, 7]
    clean = torch.from_numpy(np.stack([road_frame(H, W, seed=90 + b) for b in range(B)]))
    syn = FogSynthesizer(level="medium", seed=11, rain_p=0.002, device=cuda, filters=False)
    frames = syn.synthesize_batch(clean.to(cuda))
    flat = weights.synthetic_weights(2, seed=0)
    eng = YoloEngine(2, flat, B, (H, W), imgsz=1280, device=cuda, dtype="fp8",
                     classes_keep=keep)
    lb = eng.letterbox(frames)
    eng.calibrate(lb)
    raw = torch.empty((B, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb, raw, candidates=False)
    one = torch.empty((1, 84, eng.A), dtype=torch.float32, device=cuda)
    eng.forward_raw(lb[9:10].clone(), one, candidates=False)
    torch.cuda.synchronize()
    assert torch.equal(raw[9], one[0]), "fp8 batch-16 frame differs from the same frame alone"
    dets, n = eng.nms_from_raw(raw)
    dets, n = dets.cpu().numpy(), n.cpu().numpy()
    ref_d = yolo_ref.postprocess(raw.cpu().numpy(), (H, W), (H, W), classes_keep=keep)
    for b in range(B):
        np.testing.assert_array_equal(dets[b, :n[b]], ref_d[b].astype(np.float32).reshape(-1, 6))
    d8, n8 = eng.run_letterboxed(lb)
    d8, n8 = d8.cpu().numpy(), n8.cpu().numpy()
    scales = {bb[0]: s for bb, s in zip(eng.buffers(B), eng.act_scales)}
    pick = [0, 9]
    x = yolo_ref.preprocess(lb[pick].cpu().numpy())
    ref8 = yolo_ref.postprocess(
        yolo_ref.YoloRef(2, flat, quant="fp8", scales=scales).forward(x).numpy(), (H, W), (H, W),
        classes_keep=keep)
    ref32 = yolo_ref.postprocess(yolo_ref.YoloRef(2, flat).forward(x).numpy(), (H, W), (H, W),
                                 classes_keep=keep)
    got = [d8[b, :n8[b]] for b in pick]
    (h1, t1), (h2, t2) = _match(ref8, got), _match(got, ref8)
    (k2, m2) = _match(got, ref32, 0.5)
    print(f"config5 fp8 b16: vs fp8 oracle (IoU 0.9) {h1}/{t1}, {h2}/{t2}; GPU dets with an fp32 "
          f"match (IoU 0.5) {k2}/{m2}; detections per frame {n8.tolist()}")
    assert t1 > 0 and t2 > 0
    assert h1 >= 0.9 * t1 and h2 >= 0.9 * t2
    assert k2 >= 0.8 * m2
    eng.close()
