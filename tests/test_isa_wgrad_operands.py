"""ISA regression check of the weight-gradient staging fix ("The k_wgrad_rect zeros"):
no operand register of an in-flight staging load is rewritten inside the step loop, in any k_wgrad_rect
instantiation of the gfx950 build (tools/check_wgrad_operands.py; hipcc cross-compiles, no GPU needed)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not installed")
def test_wgrad_staging_operands_never_rewritten():
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "check_wgrad_operands.py")],
                       capture_output=True, text=True, timeout=600)
    lines = [l for l in r.stdout.splitlines() if "k_wgrad_rect" in l]
    assert len(lines) == 37, r.stdout + r.stderr  # 3 precisions x 6 shapes + 19 with fp16 operands
    assert all("foreign writes 0" in l for l in lines), r.stdout
    assert all("operand regs   0" not in l for l in lines), r.stdout  # the pinned loads were found
    assert r.returncode == 0, r.stdout + r.stderr
