"""Bit-for-bit A/B of the fused stem between two library builds: X1 and the
fused model.2.cv1 output of the production forward (stem_x1 on) for a few
frame shapes, dumped by each build (RV_LIB_VARIANT) and compared.
  python tools/stem_ab_check.py dump out_a.npz      (under RV_LIB_VARIANT=a)
  python tools/stem_ab_check.py compare out_a.npz out_b.npz"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "road-vision-system_amd"))

SHAPES = [(1080, 1920, 3), (720, 1280, 2), (480, 854, 2), (333, 500, 1), (640, 640, 2)]


def dump(path):
    import torch
    from rvs_amd import _lib
    from rvs_amd.detect import weights
    from rvs_amd.detect.yolo_hip import YoloEngine
    lib = _lib.load()
    out = {}
    for H, W, B in SHAPES:
        g = torch.Generator().manual_seed(H * 7 + W)
        fr = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, generator=g).cuda()
        eng = YoloEngine(0, weights.synthetic_weights(0, seed=3), B, (H, W), device="cuda")
        lb = eng.letterbox(fr)
        eng.set_stem_x1(True)
        eng.forward_raw(lb)
        torch.cuda.synchronize()
        ws = eng.ws.cpu().numpy()
        for i in range(lib.rv_yolo_num_buffers(eng._h)):
            info = (ctypes.c_int * 4)()
            off = ctypes.c_size_t()
            lib.rv_yolo_buffer_info(eng._h, B, i, info, ctypes.byref(off))
            h, w, c, f32 = info[0], info[1], info[2], info[3]
            if i == 1 or (c == 48 and not f32 and i <= 3):
                cs = 32 if c == 48 else c  # the fused model.2 concat holds [y0 | y1]
                n = B * h * w * cs
                out[f"{H}x{W}_buf{i}"] = ws[off.value:off.value + 2 * n].view(np.uint16).copy()
        eng.close()
    np.savez(path, **out)
    print("dumped", len(out), "arrays to", path)


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        same = np.array_equal(A[k], Bz[k])
        print(f"{k:24s} {A[k].size:>10d} {'identical' if same else 'DIFFER'}")
        bad += not same
    print("ALL IDENTICAL" if not bad else f"{bad} arrays differ")
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
