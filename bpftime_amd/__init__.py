"""bpftime_amd: MI355X-native per-packet eBPF execution path.

A drop-in for bpftime's VM C ABI (vm/vm-core/include/ebpf-vm.h) backed by a
gfx950 HIP interpreter kernel, plus device-resident maps behind the
bpftime_shm-style map / prog / link API.  See DESIGN.md.
"""
__all__ = ["isa", "programs", "gen"]
