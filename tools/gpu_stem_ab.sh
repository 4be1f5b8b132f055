set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06l}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_yolo_layers_gpu.py tests/test_detect_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RV_LIB_VARIANT=base timeout -k 10 300 python -u tools/stem_ab_check.py dump $O/base.npz && \
timeout -k 10 300 python -u tools/stem_ab_check.py dump $O/new.npz && \
python tools/stem_ab_check.py compare $O/base.npz $O/new.npz && rm -f $O/*.npz && \
TAG=${TAG:-r06l}/cv ROUNDS=2 VARS="default base" PICK="model.0 |model.2.cv2" bash tools/gpu_conv_variants.sh
