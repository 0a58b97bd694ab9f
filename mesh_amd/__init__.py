"""MI355X-native point-to-mesh spatial search for psbody-mesh.

Drop-in modules (same names as the reference's ``psbody.mesh.*``):
  ``mesh_amd.spatialsearch``  aabbtree_compute / aabbtree_nearest / aabbtree_nearest_alongnormal /
                              aabbtree_intersections_indices
  ``mesh_amd.aabb_normals``   aabbtree_n_compute / aabbtree_n_nearest / aabbtree_n_selfintersects
  ``mesh_amd.visibility``     visibility_compute
  ``mesh_amd.search``         AabbTree / AabbNormalsTree / ClosestPointTree / CGALClosestPointTree
  ``mesh_amd.mesh``           Mesh facade with the search / visibility methods
All compute runs in ``mesh_amd/lib/libmeshsearch.so`` (gfx950 HIP kernels behind a C ABI,
``include/meshsearch.h``); importing the package does not touch the GPU.
"""
__version__ = "0.1.0"
