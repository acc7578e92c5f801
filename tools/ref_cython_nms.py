#!/usr/bin/env python3
"""Build and import the REFERENCE's own ``lib/utils/cython_nms.pyx`` (container only).

SURVEY.md Appendix A step 1: the .pyx does not compile unmodified under
Cython 3 + numpy 2 because numpy 2's ``__init__.pxd`` dropped the ``np.int_t``
ctypedef (``cython_nms.pyx:45,48``) and the ``np.int`` Python alias
(``:49``).  The build substitutes exactly two tokens in a scratch copy under
/tmp -- ``np.int_t`` -> ``np.intp_t`` and ``dtype=np.int)`` -> ``dtype=np.intp)``
-- which name the same 64-bit signed integer on Linux x86-64 (``npy_long`` ==
``npy_intp``), so the compiled NMS computes what the reference's did.  Nothing
else in the file is touched, nothing is written under /root/reference, and
neither the scratch copy nor the built module enters this repository: only the
golden vectors generated with it (tests/golden/nms.npz and the fixtures of
tools/gen_goldens.py) are committed.

``load_bbox()`` builds the reference's ``lib/utils/cython_bbox.pyx`` the same way
(unmodified: it names only ``np.float32_t``) for box voting's ``bbox_overlaps``.

Usage: ``from tools.ref_cython_nms import load; cy = load(); cy.nms(dets, thr)``
"""
import hashlib
import importlib.util
import os
import sys
import tempfile

REF_PYX = "/root/reference/lib/utils/cython_nms.pyx"
REF_BBOX_PYX = "/root/reference/lib/utils/cython_bbox.pyx"
SUBS = (("np.int_t", "np.intp_t"), ("dtype=np.int)", "dtype=np.intp)"))


def _scratch_dir(src: str, name: str) -> str:
    tag = hashlib.sha1(src.encode()).hexdigest()[:12]
    return os.path.join(tempfile.gettempdir(), "vosdet_%s_%s" % (name, tag))


def load():
    """Return the compiled reference cython_nms module (builds once per source hash)."""
    return _build(REF_PYX, "ref_cython_nms", SUBS)


def load_bbox():
    """Return the compiled reference cython_bbox module (source unmodified)."""
    return _build(REF_BBOX_PYX, "ref_cython_bbox", ())


def _build(path, name, subs):
    with open(path) as f:
        src = f.read()
    patched = src
    for a, b in subs:
        assert a in patched, "reference text changed: %r not found" % a
        patched = patched.replace(a, b)
    d = _scratch_dir(src, name)
    os.makedirs(d, exist_ok=True)
    built = [f for f in os.listdir(d) if f.startswith(name) and f.endswith(".so")]
    if not built:
        pyx = os.path.join(d, name + ".pyx")
        with open(pyx, "w") as f:
            f.write(patched)
        import numpy
        from Cython.Build import cythonize
        from setuptools import Extension
        from setuptools.dist import Distribution
        ext = Extension(name, [pyx], include_dirs=[numpy.get_include()],
                        extra_compile_args=["-O2"])
        dist = Distribution({"ext_modules": cythonize([ext], language_level=3, quiet=True)})
        cmd = dist.get_command_obj("build_ext")
        cmd.inplace = False
        cmd.build_lib = d
        cmd.build_temp = os.path.join(d, "tmp")
        dist.run_command("build_ext")
        built = [f for f in os.listdir(d) if f.startswith(name) and f.endswith(".so")]
    spec = importlib.util.spec_from_file_location(name, os.path.join(d, built[0]))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


if __name__ == "__main__":
    import numpy as np
    cy = load()
    d = np.array([[0, 0, 9, 9, .9], [0, 0, 9, 4, .8], [20, 20, 30, 30, .7]], np.float32)
    print(cy.nms(d, np.float32(0.5)))
    sys.exit(0)
