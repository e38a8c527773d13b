"""antidote_amd — MI355X-native engine for AntidoteDB's snapshot materialization path.

The product is the C-ABI library antidote_amd/libantidote_gpu.so (HIP kernels
for gfx950 + host engine, include/antidote_gpu.h).  This package is the
host-side mirror of the reference's Erlang interface above that ABI:

  clocksi_materializer  materialize/4, materialize_eager/3, new/1
  materializer          update_snapshot/3, belongs_to_snapshot_op/3
  materializer_vnode    read/update/store_ss over a device-resident op log
  stable_time_functions get_min_time/1, update_func_min/2 (+ RCCL exchange)
  vector_orddict        get_smaller/2 on device

Importing the package loads nothing; the first engine call loads the
library and raises EngineUnavailable if it (or a GPU) is missing — there is
no CPU fallback.
"""
from ._abi import ABI_VERSION  # noqa: F401

__all__ = ["ABI_VERSION"]
