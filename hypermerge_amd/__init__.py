"""hypermerge_amd — MI355X-native batched CRDT merge for hypermerge's remote-change path.

The product is the HIP library (csrc/, built to _lib/libhmgpu.so) behind the
C-ABI of include/hypermerge_amd.h; this package holds its host-side mirror of
the reference interface (columnar encoder, clocks, DocBackend contract) and
the ctypes binding.  See DESIGN.md.
"""
__all__ = ["columnar", "clock", "engine", "render", "synth"]
