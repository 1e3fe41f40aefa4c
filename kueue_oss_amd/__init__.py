"""kueue_oss_amd — MI355X-native Topology-Aware Scheduling evaluation.

A from-scratch HIP/CDNA4 implementation of Kueue's TAS evaluation path
(``TASFlavorSnapshot.FindTopologyAssignmentsForFlavor``, reference
pkg/cache/scheduler/tas_flavor_snapshot.go:519) behind a C-ABI
(include/kueue_tas.h).  See DESIGN.md.
"""
from .native import (  # noqa: F401
    NativeLibraryMissing,
    TASFlavorSnapshot,
    build_native,
    library_path,
    load_library,
)

__all__ = ["TASFlavorSnapshot", "NativeLibraryMissing", "build_native", "library_path", "load_library"]
