"""CPU oracle for the FoundationStereo cost-volume + refinement hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this package, and only as the
checker / the timed CPU baseline -- never as the thing measured or shipped.
The product path (``foundationstereo_amd``) never imports it and fails loudly
when its HIP library is missing.

Parity pin: the restatement is checked against golden vectors generated in
the build container by importing the reference modules
(``tools/make_goldens.py`` -> ``tests/golden/*.npz``); see DESIGN.md §Oracle.
"""
from .stereo_oracle import *  # noqa: F401,F403
