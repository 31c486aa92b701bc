"""The host-to-device paths give the same bytes: the upload ring's copy
kernel over fine-grained mapped pinned memory (default), over non-coherent
mapped memory and hipMemcpyAsync (DPF_AMD_UPLOAD), one EvaluateAt call's
points copied instead of read in place (DPF_AMD_ZERO_COPY=0) and its key
part uploaded instead of host-written into fine-grained VRAM
(DPF_AMD_HOST_WRITE=0).  Each variant runs tests/upload_paths_case.py in a
child process (the knobs are read once per process); the default paths are
the ones every other GPU test checks against the oracle."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CASE = os.path.join(HERE, "upload_paths_case.py")
VARIANTS = [{}, {"DPF_AMD_HOST_WRITE": "0"}, {"DPF_AMD_ZERO_COPY": "0"},
            {"DPF_AMD_UPLOAD": "sdma"}, {"DPF_AMD_UPLOAD": "kernel"}]


def _run(extra):
    env = dict(os.environ)
    env.update(extra)
    r = subprocess.run([sys.executable, CASE], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_run():
    return _run({})


@pytest.mark.gpu
@pytest.mark.parametrize("extra", VARIANTS[1:], ids=lambda e: ",".join("%s=%s" % kv for kv in e.items()))
def test_upload_variants_equal_default(default_run, extra):
    assert _run(extra) == default_run
