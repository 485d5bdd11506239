"""oracle — CPU restatement of the reference's hot path, used ONLY as the checker.

TEST INFRASTRUCTURE. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything under oracle/. The product (robust-audio-deepfake-evolution_amd/) never imports it and has
no CPU fallback.

Each function cites the reference file:line it restates (reference = lux-liang/Robust-Audio-Deepfake-
Evolution, mounted read-only at /root/reference in the build container only). The restatement is
pinned by golden vectors in tests/golden/, generated from the reference itself in the build container
by tests/golden/make_golden.py (see DESIGN.md "Oracle and parity"). Third-party arithmetic the
reference calls but that is absent from the image (mamba_ssm CUDA kernels, peft, kornia, torchaudio)
is restated from its published algorithm and marked "parity unpinned" where no reference-owned
fixture covers it.
"""
