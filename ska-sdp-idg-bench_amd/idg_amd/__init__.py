"""idg_amd -- MI355X-native IDG gridder/degridder (host side).

A Python mirror of the reference's gridder/degridder operator interface over
the C ABI of libidg_mi355x.so (include/idg_mi355x.h).  Importing this package
loads the HIP library and raises if it is missing: there is no CPU fallback.
"""
from .api import (IMAGE_SIZE, METADATA_DTYPE, NR_CORRELATIONS, W_STEP,
                  IdgError, abi_version, adder_launch, as_metadata,
                  bytes_gridder, c_run_degridder, c_run_gridder,
                  degrid_from, degridder_launch, device_name, flops_gridder,
                  generate, grid_onto, gridder_fft_launch, gridder_launch,
                  host_chunk_plan,
                  kernel_name,
                  nr_subgrids_for, precision_options, p_run_degridder, p_run_gridder,
                  release_workspaces,
                  splitter_fft_launch, splitter_launch, subgrid_fft_launch,
                  validate_metadata)
from ._lib import LIB_PATH
from . import shard

__all__ = [
    "IMAGE_SIZE", "METADATA_DTYPE", "NR_CORRELATIONS", "W_STEP", "IdgError",
    "abi_version", "adder_launch", "as_metadata", "bytes_gridder",
    "c_run_degridder", "c_run_gridder", "degrid_from", "degridder_launch",
    "device_name", "flops_gridder", "generate", "grid_onto",
    "gridder_fft_launch", "gridder_launch", "host_chunk_plan", "kernel_name", "nr_subgrids_for", "p_run_degridder",
    "precision_options", "release_workspaces",
    "p_run_gridder", "splitter_fft_launch", "splitter_launch",
    "subgrid_fft_launch",
    "validate_metadata", "LIB_PATH", "shard",
]
