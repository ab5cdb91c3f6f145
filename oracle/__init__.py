"""CPU oracle for the CCMM shadow-rate BVAR-SV Gibbs sweep.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the package
``ccmmshadowratevar-code_amd/`` and ``libccmm.so``) may import, call or
link anything under ``oracle/``.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg use it, and only as the checker.

PARITY UNPINNED: the reference is MATLAB (no MATLAB/Octave in this image)
and ships no tests, golden vectors or fixtures; its SV sampler lives in the
absent ``em-matlabbox`` submodule.  See ``ccmm_oracle.py`` header.
"""
