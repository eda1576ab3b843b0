"""sfa_hip — MI355X-native (gfx950) runtime for the SFA3D FPN-ResNet-18 hot path.

Layers:
  _lib       ctypes binding of libsfa_hip.so (include/sfa_hip.h); no CPU fallback.
  runtime    weight packing, KfpnEngine (forward), BevVoxelizer, Decoder,
             DetectorPipeline (fixed-shape BEV -> forward -> decode, HIP-graph capturable).
  synthetic  deterministic weights / BEV tensors / point clouds (no dataset offline).
  dist       frame-sharded multi-GPU helpers (one process per GPU, RCCL gather).

The reference-compatible modules (``models``, ``utils``, ``data_process``,
``config``) live next to this package under the same ``sfa`` root, mirroring
the reference's import paths.
"""

from ._lib import SfaNativeError, lib  # noqa: F401

__all__ = ["SfaNativeError", "lib"]
