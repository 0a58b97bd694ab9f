"""Drop-in for ``psbody.mesh.serialization``'s two native readers: ``loadobj``
(mesh/src/py_loadobj.cpp) and ``plyutils.read`` (mesh/src/plyutils.c over rply.c), backed by the
memory-mapped parsers of libmeshsearch (mesh_amd/csrc/loaders.cpp).  Writers and the pure-Python
serialisation helpers of the reference are out of scope (they do not feed the search path)."""
