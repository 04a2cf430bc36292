"""arpc_amd -- MI355X-native batched Symphony codec for aRPC's serializer hot path.

Layers:
  include/symphony_hip.h      C ABI (the drop-in boundary; cgo binds it)
  arpc_amd/csrc/*.hip         gfx950 encode / decode kernels + C-ABI implementation
  arpc_amd/_native.py         ctypes binding of that ABI (no CPU fallback)
  arpc_amd/codec.py           device-resident batched API over torch tensors
  arpc_amd/serializer.py      mirror of pkg/serializer (Serializer / SymphonySerializer)
  arpc_amd/schemas.py         the flat schemas on the hot path (KV, echo)
  arpc_amd/datagen.py         seeded synthetic batches (tests, bench)
"""
from . import schemas  # noqa: F401

__all__ = ["schemas"]
