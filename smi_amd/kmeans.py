"""Host mirror of kmeans_smi (examples/host/kmeans_smi.cpp,
examples/kernels/kmeans_smi.cl).

The reference host generates Gaussian blobs on rank 0, MPI_Bcasts the
initial centroids and MPI_Scatters the points (kmeans_smi.cpp:96-166); the
device program then iterates assign / accumulate / SMI_Reduce / SMI_Bcast /
divide.  Here every rank holds its points and the initial centroids in
device memory and one call runs all iterations through the C ABI
(include/smi/kmeans.h); `assign` and `accumulate` expose the two halves.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .comm import Comm

# reference build configuration (examples/CMakeLists.txt:4-11)
REFERENCE_WIDTH = 16     # SMI_VECTORIZATION_WIDTH
REFERENCE_DIMS = 64      # SMI_KMEANS_DIMS
REFERENCE_CLUSTERS = 8   # SMI_KMEANS_CLUSTERS
REFERENCE_RANKS = 8      # SMI_KMEANS_RANKS


def _check(t: torch.Tensor, dtype, name: str) -> None:
    if t.dtype != dtype or not t.is_contiguous() or not t.is_cuda:
        raise _lib.SMIError(f"{name} must be a contiguous {dtype} device tensor")


def assign(points: torch.Tensor, centroids: torch.Tensor, width: int = REFERENCE_WIDTH,
           out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """ComputeDistance (kmeans_smi.cl:36-88): the cluster of every point."""
    _check(points, torch.float32, "points")
    _check(centroids, torch.float32, "centroids")
    n, dims = points.shape
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=points.device)
    _lib.call("smi_kmeans_assign", points.data_ptr(), n, dims, centroids.data_ptr(), centroids.shape[0],
              width, out.data_ptr(), _lib.stream_handle(stream))
    return out


def accumulate(points: torch.Tensor, assignment: torch.Tensor, clusters: int,
               sums: torch.Tensor | None = None, counts: torch.Tensor | None = None,
               stream=None) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-cluster sums (fp32 chains in point order) and counts
    (kmeans_smi.cl:113-127)."""
    _check(points, torch.float32, "points")
    _check(assignment, torch.int32, "assignment")
    n, dims = points.shape
    if sums is None:
        sums = torch.empty((clusters, dims), dtype=torch.float32, device=points.device)
    if counts is None:
        counts = torch.empty(clusters, dtype=torch.int32, device=points.device)
    _lib.call("smi_kmeans_accumulate", points.data_ptr(), n, dims, assignment.data_ptr(), clusters,
              sums.data_ptr(), counts.data_ptr(), _lib.stream_handle(stream))
    return sums, counts


def kmeans(comm: Comm, points: torch.Tensor, centroids: torch.Tensor, iterations: int,
           width: int = REFERENCE_WIDTH, stream=None) -> torch.Tensor:
    """The kmeans_smi program on this rank's points; `centroids` is updated
    in place (the same final centroids on every rank) and returned."""
    _check(points, torch.float32, "points")
    _check(centroids, torch.float32, "centroids")
    n, dims = points.shape
    _lib.call("smi_kmeans", comm.handle, points.data_ptr(), n, dims, centroids.shape[0], width,
              centroids.data_ptr(), iterations, _lib.stream_handle(stream))
    return centroids


def split_points(points: np.ndarray, size: int, rank: int) -> np.ndarray:
    """MPI_Scatter of kmeans_smi.cpp:165-166: equal contiguous shares."""
    if len(points) % size:
        raise ValueError("Number of points must be divisible by number of ranks.")  # kmeans_smi.cpp:75-77
    per = len(points) // size
    return points[rank * per:(rank + 1) * per]


def synthetic_points(num_points: int, clusters: int = REFERENCE_CLUSTERS, dims: int = REFERENCE_DIMS,
                     seed: int = 5, device=None) -> tuple[torch.Tensor, torch.Tensor]:
    """Data built like kmeans_smi.cpp:99-147 (with torch's generator, not the
    reference's std::default_random_engine): cluster means uniform in
    [-5, 5), point i drawn from N(mean_{i % clusters}, 1), initial centroids
    = `clusters` random points."""
    g = torch.Generator(device=device or "cpu").manual_seed(seed)
    kw = dict(device=device, generator=g)
    means = torch.rand((clusters, dims), **kw) * 10 - 5
    pts = torch.randn((num_points, dims), **kw)
    pts += means[torch.arange(num_points, device=device) % clusters]
    pick = torch.randint(0, num_points, (clusters,), **kw)
    return pts, pts[pick].clone()
