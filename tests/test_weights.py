"""Loading real Ultralytics checkpoints (a4: YOLO(model) + model.fuse(),
src/detect/yolo_ultralytics.py:16-17) -- CPU only.

No real yolov8n weights exist here (.MISSING_LARGE_BLOBS:1), so a synthetic
Ultralytics-format state_dict is built: unfused Conv blocks
(``model.N.conv.weight`` + ``model.N.bn.{weight,bias,running_mean,
running_var,num_batches_tracked}``), the Detect head's plain convs
(``model.22.cv2.i.2.weight/.bias``) and the DFL conv.  Checks:
  * the fold equals fuse_conv_and_bn's arithmetic (BatchNorm2d eps 1e-3):
    bit for bit against the exact float32 products torch.mm(diag(scale), w)
    denotes, and within 1 ulp of torch.mm itself -- the CPU BLAS behind
    torch.mm (MKL here) returns 1-ulp-different values for some elements of
    a diagonal-matrix product, so its bits are platform-dependent;
  * the folded network equals the UNFUSED torch network (conv -> BN eval ->
    SiLU, oracle YoloRef.from_unfused) end to end within fp32 rounding;
  * the fused state_dict form (conv.bias, after model.fuse()) and the
    safetensors / npz / weights-only torch formats load to the same weights;
  * the plan's own key names (round-1 files) still load."""
import numpy as np
import pytest
import torch

from oracle import yolo_ref


def _unfused_state_dict(variant=0, seed=0):
    from rvs_amd.detect.weights import conv_list, synthetic_weights
    flat = synthetic_weights(variant, seed)
    rng = np.random.default_rng(seed + 1)
    sd, off = {}, 0
    for name, cin, cout, k, s, act in conv_list(variant):
        nw = cout * cin * k * k
        wf = flat[off:off + nw].reshape(cout, cin, k, k)
        bf = flat[off + nw:off + nw + cout]
        off += nw + cout
        if act:  # Conv block: un-fold the calibrated weights into conv + BN
            gamma = rng.uniform(0.5, 1.5, cout).astype(np.float32)
            var = rng.uniform(0.5, 2.0, cout).astype(np.float32)
            mean = rng.normal(0, 0.1, cout).astype(np.float32)
            sd_ = np.sqrt(var + np.float32(1e-3))
            scale = gamma / sd_
            sd[name + ".conv.weight"] = (wf / scale[:, None, None, None]).astype(np.float32)
            sd[name + ".bn.weight"] = gamma
            sd[name + ".bn.bias"] = (bf + gamma * mean / sd_).astype(np.float32)
            sd[name + ".bn.running_mean"] = mean
            sd[name + ".bn.running_var"] = var
            sd[name + ".bn.num_batches_tracked"] = np.array(1000, np.int64)
        else:
            sd[name + ".weight"] = wf.copy()
            sd[name + ".bias"] = bf.copy()
    sd["model.22.dfl.conv.weight"] = np.arange(16, dtype=np.float32).reshape(1, 16, 1, 1)
    return sd


def _torch_fuse(w, gamma, beta, mean, var, eps=1e-3, exact=False):
    """ultralytics.utils.torch_utils.fuse_conv_and_bn's arithmetic; exact=True
    evaluates the diagonal matmuls as the exact float32 products they denote."""
    w, gamma, beta = torch.from_numpy(w), torch.from_numpy(gamma), torch.from_numpy(beta)
    mean, var = torch.from_numpy(mean), torch.from_numpy(var)
    wc = w.view(w.shape[0], -1)
    scale = gamma.div(torch.sqrt(eps + var))
    w_bn = torch.diag(scale)
    fw = (scale[:, None] * wc if exact else torch.mm(w_bn, wc)).view(w.shape)
    b_conv = torch.zeros(w.shape[0])
    b_bn = beta - gamma.mul(mean).div(torch.sqrt(var + eps))
    fb = (scale * b_conv if exact else torch.mm(w_bn, b_conv.reshape(-1, 1)).reshape(-1)) + b_bn
    return fw.numpy(), fb.numpy()


def test_fold_matches_torch_fuse_conv_and_bn_bitwise():
    from rvs_amd.detect.weights import conv_list, flat_from_state_dict
    sd = _unfused_state_dict()
    flat = flat_from_state_dict(sd, 0)
    off = 0
    for name, cin, cout, k, s, act in conv_list(0):
        nw = cout * cin * k * k
        w, b = flat[off:off + nw].reshape(cout, cin, k, k), flat[off + nw:off + nw + cout]
        off += nw + cout
        if act:
            args = [sd[name + x] for x in (".conv.weight", ".bn.weight", ".bn.bias",
                                           ".bn.running_mean", ".bn.running_var")]
            fw, fb = _torch_fuse(*args, exact=True)
            np.testing.assert_array_equal(w, fw, err_msg=name)
            np.testing.assert_array_equal(b, fb, err_msg=name)
            mw, mb = _torch_fuse(*args)  # torch.mm: within 1 ulp
            np.testing.assert_array_max_ulp(w, mw, maxulp=1)
            np.testing.assert_array_max_ulp(b, mb, maxulp=1)
        else:
            np.testing.assert_array_equal(w, sd[name + ".weight"])
    assert off == flat.size


def test_folded_network_equals_unfused_network():
    from rvs_amd.detect.weights import flat_from_state_dict
    sd = _unfused_state_dict()
    x = torch.rand(1, 3, 128, 160, generator=torch.Generator().manual_seed(0))
    ref = yolo_ref.YoloRef.from_unfused(0, sd).forward(x).numpy()
    got = yolo_ref.YoloRef(0, flat_from_state_dict(sd, 0)).forward(x).numpy()
    # fp32 rounding of the fold (BN folded into the weights vs applied after
    # the conv) only; the synthetic network amplifies it (measured: class
    # score |d| 1.1e-4 at p99.9, 2.2e-4 worst; box 0.008 px at p99, 0.13 px
    # worst)
    ds = np.abs(got[:, 4:] - ref[:, 4:])
    db = np.abs(got[:, :4] - ref[:, :4])
    assert np.percentile(ds, 99.9) < 5e-4 and ds.max() < 2e-3
    assert np.percentile(db, 99) < 0.05 and db.max() < 0.5


def test_checkpoint_formats_and_fused_keys(tmp_path):
    from safetensors.numpy import save_file
    from rvs_amd.detect.weights import conv_list, flat_from_state_dict, load_weights
    sd = _unfused_state_dict()
    want = flat_from_state_dict(sd, 0)
    save_file({k: np.ascontiguousarray(v) for k, v in sd.items()}, str(tmp_path / "n.safetensors"))
    np.savez(tmp_path / "n.npz", **sd)
    torch.save({"model." + k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()},
               tmp_path / "n.pt")  # YOLO(...).state_dict() nesting
    for f in ("n.safetensors", "n.npz", "n.pt"):
        np.testing.assert_array_equal(load_weights(str(tmp_path / f), 0), want, err_msg=f)
    # after model.fuse(): Conv blocks carry conv.bias, no bn.*
    fused, plan, off = {}, {}, 0
    for name, cin, cout, k, s, act in conv_list(0):
        nw = cout * cin * k * k
        w, b = want[off:off + nw].reshape(cout, cin, k, k), want[off + nw:off + nw + cout]
        off += nw + cout
        fused[name + (".conv.weight" if act else ".weight")] = w
        fused[name + (".conv.bias" if act else ".bias")] = b
        plan[name + ".weight"], plan[name + ".bias"] = w, b
    np.testing.assert_array_equal(flat_from_state_dict(fused, 0), want)
    np.testing.assert_array_equal(flat_from_state_dict(plan, 0), want)


def test_missing_keys_raise():
    from rvs_amd.detect.weights import flat_from_state_dict
    sd = _unfused_state_dict()
    del sd["model.4.m.1.cv2.conv.weight"]
    with pytest.raises(KeyError, match="model.4.m.1.cv2"):
        flat_from_state_dict(sd, 0)
