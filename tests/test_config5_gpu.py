"""BASELINE config 5: YOLOv8m at 1280x1280, batch 16, on fog/rain-augmented
frames made on the device (rv_fog_rain_u8).

Computed in bf16 (the fp8 MFMA variant of config 5 is not built yet; see
DESIGN.md).  Checks:
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
