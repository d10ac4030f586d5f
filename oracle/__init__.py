"""ORACLE -- test infrastructure only.

A CPU (torch fp32, eager ATen on the host) restatement of the reference
video-generation/diffusion denoising path of wdas03/lipreading-video-generation,
written functionally over plain parameter dicts keyed by the reference
state-dict names.  Each function cites the reference file:line it restates.

Pinned against golden vectors produced by importing the reference modules in
the build container (tests/golden/gen_golden.py -> tests/golden/*.npz);
tests/test_oracle_golden.py checks every fixture.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product path (lipreading-video-generation_amd/) never
does: it runs on libvdiff.so or raises.
"""
