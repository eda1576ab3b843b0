"""CPU oracle — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the reference algorithms of the hot path so
the HIP implementation can be checked against them.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything from here, and only as the checker / the reported CPU baseline.  The
product path (``lidar-image_object-detection_-fpn_resnet-yolov8_amd/``) never
imports it and fails loudly when the HIP library is missing.

Pinning: every restatement here is checked against the golden fixtures in
``tests/golden/`` which were produced by running the reference's own Python
functions in the build container (``tests/golden/gen_golden.py``), see
``tests/test_oracle_golden.py``.

Modules
  bev_oracle     get_filtered_lidar + makeBEVMap  (numpy; kitti_data_utils.py:228-251,
                 kitti_bev_utils.py:22-55)
  bev_oracle.c   the same in plain C (fast single-thread CPU baseline for BEV)
  model_oracle   PoseResNet / KFPN forward in torch fp32 on CPU (fpn_resnet.py:37-301)
  decode_oracle  _sigmoid/_nms/_topk/decode/post_processing/convert_det_to_real_values
                 (torch_utils.py:44-45, evaluation_utils.py:21-193)
"""
