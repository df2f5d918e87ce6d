"""tools/isa_vmcheck.py: the build's check of the counted LDS-DMA waits (RRIN_VMWAIT) on the
gfx950 ISA -- a synthetic listing for the path logic, then the real kind-6 tile compiled with the
scheduler that broke it in round 5 (max-ilp), with and without the vm_fence()s."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import isa_vmcheck  # noqa: E402

HEAD = """\t.type\tk,@function
k:  ; @k
"""
TAIL = """\ts_endpgm
.Lfunc_end0:
"""
DMA = "\tbuffer_load_dwordx4 v1, s[0:3], 0 offen lds\n"
LD = "\tbuffer_load_dwordx4 v[4:7], v1, s[4:7], 0 offen\n"
ST = "\tbuffer_store_dwordx4 v[4:7], v1, s[4:7], 0 offen\n"


def wait(n, lds, ld):
    return f"\t;;#ASMSTART\n\ts_waitcnt vmcnt({n}) ; rrin-vm lds={lds} ld={ld}\n\t;;#ASMEND\n"


def run(tmp_path, body):
    p = tmp_path / "k.s"
    p.write_text(HEAD + body + TAIL)
    return isa_vmcheck.check_file(str(p))


def test_declared_order_passes(tmp_path):
    # raw(0), U x2, raw(1), U x2; wait for raw(0): 4 register loads and 1 DMA younger
    assert run(tmp_path, DMA + LD + LD + DMA + LD + LD + wait(5, 1, 4)) == (1, 0)


def test_load_moved_across_dma_fails(tmp_path):
    # reordering among the younger loads keeps the composition, and the wait stays right
    assert run(tmp_path, DMA + LD + LD + LD + DMA + LD + wait(5, 1, 4)) == (1, 0)
    # raw(0) issued after a U load: the 5 youngest now hold both DMAs -- vmcnt(5) could pass with
    # raw(0) in flight
    assert run(tmp_path, LD + DMA + LD + DMA + LD + LD + wait(5, 1, 4)) == (1, 1)


def test_stores_are_skipped(tmp_path):
    assert run(tmp_path, DMA + LD + ST + ST + LD + wait(2, 0, 2)) == (1, 0)


def test_undeclared_counted_wait_fails(tmp_path):
    body = DMA + LD + "\t;;#ASMSTART\n\ts_waitcnt vmcnt(1)\n\t;;#ASMEND\n"
    assert run(tmp_path, body) == (1, 1)
    # vmcnt(0) needs no declaration
    assert run(tmp_path, DMA + LD + "\t;;#ASMSTART\n\ts_waitcnt vmcnt(0)\n\t;;#ASMEND\n") == (0, 0)


def test_short_path_from_entry_fails(tmp_path):
    assert run(tmp_path, LD + wait(2, 0, 2)) == (1, 1)


def test_every_path_through_a_loop(tmp_path):
    # prologue: raw, U; loop: wait (covers the raw), U, raw; back edge.  From the prologue the
    # youngest load is the U; around the back edge it is the raw issued last in the loop body
    body = (DMA + LD + ".LBB0_1:\n" + wait(1, 0, 1) + LD + DMA + "\ts_cbranch_scc1 .LBB0_1\n")
    assert run(tmp_path, body) == (1, 1)
    body = (DMA + LD + ".LBB0_1:\n" + wait(1, 0, 1) + DMA + LD + "\ts_cbranch_scc1 .LBB0_1\n")
    assert run(tmp_path, body) == (1, 0)


HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("python3") is None, reason="needs hipcc")
@pytest.mark.parametrize("fenced", [False, True])
def test_kind6_tile_under_max_ilp(tmp_path, fenced):
    """Round 5's failing build: conv_winoc.hip under -amdgpu-sched-strategy=max-ilp.  Without the
    vm_fence()s the scheduler moves U loads across the raw-tile DMA and the check fails; with
    them every counted wait sees its declared loads."""
    out = tmp_path / "winoc.s"
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + os.path.join(REPO, "include"),
           "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "--cuda-device-only", "-S",
           "-mllvm", "-amdgpu-sched-strategy=max-ilp", "-o", str(out),
           os.path.join(REPO, "rrin_amd", "csrc", "conv_winoc.hip")]
    if not fenced:
        cmd.insert(1, "-DRRIN_NO_VMFENCE")
    subprocess.run(cmd, check=True, capture_output=True)
    n, failed = isa_vmcheck.check_file(str(out))
    assert n >= 10
    assert (failed == 0) == fenced, (n, failed)
