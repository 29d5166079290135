"""The reference's own unit tests (Attempt_1/test_*.py) run against the drop-in modules.

SURVEY §7 step 2 set "all reference tests must pass" as the bar for the drop-in layer. This runs them
here, in the build container, as they are: nothing is copied out of /root/reference, the reference's
directory goes to the END of sys.path (pytest --import-mode=append) so ``cuvs-rag_amd/`` supplies
``gpu_resource_manager``, ``embedding_distribution_manager``, ``index_building_coordinator`` and
``search_result_aggregator``, and no bytecode is written next to the reference files. Skipped where
/root/reference does not exist (the GPU box).

Known outcome: 131 passed, 1 skipped (its CUDA-gated integration test), and 2 failed -- both
``test_distribute_embeddings_valid`` variants, whose patched ``Tensor.to`` returns CPU tensors that
the reference's own ``validate_distribution`` rejects too.
"""
import os
import re
import subprocess
import sys

import pytest

REF = "/root/reference/Attempt_1"
PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cuvs-rag_amd")
FILES = ["test_gpu_resource_manager.py", "test_index_building_coordinator.py", "test_embedding_distribution_manager.py",
         "test_embedding_distribution_manager_fixed.py", "test_search_result_aggregator.py"]
KNOWN_FAILURES = {
    "test_embedding_distribution_manager.py::TestEmbeddingDistributionManager::test_distribute_embeddings_valid",
    "test_embedding_distribution_manager_fixed.py::TestEmbeddingDistributionManager::test_distribute_embeddings_valid",
}


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference checkout exists only in the build container")
def test_reference_unit_tests_pass_against_dropins(tmp_path):
    env = dict(os.environ, PYTHONPATH=PKG, PYTHONDONTWRITEBYTECODE="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "pytest", "--import-mode=append", "-p", "no:cacheprovider", "-q", "-rf",
           "--rootdir", REF] + [os.path.join(REF, f) for f in FILES]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    m = re.search(r"(?:(\d+) failed, )?(\d+) passed(?:, (\d+) skipped)?", out)
    assert m, out[-3000:]
    failed, passed, skipped = int(m.group(1) or 0), int(m.group(2)), int(m.group(3) or 0)
    failures = {ln.split("FAILED ", 1)[1].split(" ")[0].split("Attempt_1/")[-1]
                for ln in out.splitlines() if ln.startswith("FAILED ")}
    assert failures == KNOWN_FAILURES, out[-3000:]
    assert (passed, failed, skipped) == (131, 2, 1), out[-3000:]
    assert not any(n.endswith(".pyc") or n == "__pycache__" for n in os.listdir(REF))
