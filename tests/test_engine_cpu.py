"""Host logic of RoadVisionEngine that needs no GPU: the reference's
soft-disable of a projector / tracker that fails to build
(main_preview.py:64-78) and the clear error of detector-only entry points
when detect.enabled is false."""
import copy

import pytest


def _cfg(points):
    from rvs_amd.config import load_config
    cfg = copy.deepcopy(load_config())
    cfg["detect"]["enabled"] = False
    cfg["geometry"]["enabled"] = True
    cfg["geometry"]["projector"]["image_points"] = points
    cfg["geometry"]["projector"]["world_points"] = points
    return cfg


def test_projector_failure_warns_and_disables():
    from rvs_amd.engine import RoadVisionEngine
    with pytest.warns(UserWarning, match="at least 4 image points"):
        eng = RoadVisionEngine(_cfg([[0, 0], [1, 1]]), 2, (64, 64), device="cpu")
    assert eng.projector is None and eng.tracker is None and eng.detector is None


def test_projector_unknown_type_warns_and_disables():
    from rvs_amd.engine import RoadVisionEngine
    cfg = _cfg([[0, 0], [1, 0], [1, 1], [0, 1]])
    cfg["geometry"]["projector"]["type"] = "lidar"
    with pytest.warns(UserWarning, match="unknown projector type"):
        eng = RoadVisionEngine(cfg, 1, (32, 32), device="cpu")
    assert eng.projector is None


@pytest.mark.parametrize("call", ["step_unit", "track_stage", "track_pair_stage",
                                  "track_handback", "detect_stage", "yolo_stage", "autotune"])
def test_detector_entry_points_need_detector(call):
    from rvs_amd.engine import RoadVisionEngine
    cfg = _cfg([])
    cfg["geometry"]["enabled"] = False
    eng = RoadVisionEngine(cfg, 1, (32, 32), device="cpu")
    args = {"step_unit": ([], [], []), "track_stage": (None,), "track_pair_stage": ([], 0, []),
            "track_handback": (None, None, None, None), "detect_stage": (None,),
            "yolo_stage": (None,), "autotune": (None,)}[call]
    with pytest.raises(ValueError, match="needs the detector"):
        getattr(eng, call)(*args)
