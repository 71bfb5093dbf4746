"""flpytorch_amd — MI355X-native hot path of FL_PyTorch's simulated uplink.

* ``flpytorch_amd.aggregation`` — the drop-in plug-in surface (the reference reserves the
  empty package ``fl_pytorch/aggregation/``): ``Compressor`` / ``initCompressor`` with the
  reference's codec protocol, ``serverGradient`` reducers, the fused ``UplinkReducer`` and
  ``install()`` which rebinds them into an unchanged reference tree.
* ``flpytorch_amd.sharding`` — clients sharded over GPUs (one process per GPU, RCCL reduce).
* ``flpytorch_amd.harness`` — the round loop of §3.2 (model_funcs.py:459-614) around them.

All compute runs in ``libflcodec.so`` (HIP, gfx950); see include/flcodec.h and DESIGN.md.
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"
