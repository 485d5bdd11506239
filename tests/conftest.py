import os
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")  # see radhip/__init__.py (graph memset replay)
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "robust-audio-deepfake-evolution_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); parity tests of the HIP path")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no ROCm GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            path = os.path.join(GOLDEN, name)
            if name.endswith(".npz"):
                cache[name] = dict(np.load(path, allow_pickle=False))
            else:
                import json
                cache[name] = json.load(open(path))
        return cache[name]
    return load


REFERENCE = "/root/reference"


def reference_present():
    return os.path.isdir(REFERENCE)


@pytest.fixture(autouse=True)
def _gpu_heartbeat(request):
    """Long GPU tests (the fp32 accumulation-window test spends minutes in MIOpen's fp32 solver search
    and three model builds) print nothing while they run; a runner that takes 3 silent minutes for a
    hang would kill them. Every 45 s this writes one progress line naming the running test to the real
    stdout (capture suspended) and, on the GPU box, to gpurun_out/pytest_heartbeat.log."""
    if "gpu" not in request.keywords:
        yield
        return
    import threading
    import time
    capman = request.config.pluginmanager.getplugin("capturemanager")
    stop = threading.Event()
    t0 = time.time()
    out_dir = os.path.join(os.environ.get("GRAFT_REPO_ROOT", ROOT), "gpurun_out")

    def beat():
        while not stop.wait(45.0):
            line = f"[heartbeat] {request.node.nodeid} running {time.time() - t0:.0f} s\n"
            try:
                if os.path.isdir(out_dir):
                    with open(os.path.join(out_dir, "pytest_heartbeat.log"), "a") as f:
                        f.write(line)
                if capman is not None:
                    with capman.global_and_fixture_disabled():
                        sys.stdout.write(line)
                        sys.stdout.flush()
            except Exception:
                pass

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        yield
    finally:
        stop.set()
        th.join()
