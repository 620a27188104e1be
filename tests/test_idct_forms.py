"""CPU: the pixel kernel's IDCT forms (the dot2-chained packed row pass and
the high-half column pass, hjd_device.hpp) equal the plain restatement on
random legal blocks and the clamp-edge known answers (tools/check/idct_forms.hip,
built with hipcc for the host)."""
import os
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_idct_forms_match_restatement():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "idct_forms")
        src = os.path.join(REPO, "tools", "check", "idct_forms.hip")
        inc = [f"-I{os.path.join(REPO, 'ocljpegdecoder_amd', 'csrc')}", f"-I{os.path.join(REPO, 'include')}"]
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", *inc, src, "-o", exe],
                       check=True, capture_output=True, timeout=300)
        p = subprocess.run([exe, "60000"], capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stdout + p.stderr
        assert "mismatches 0" in p.stdout


def test_slot_map_composition():
    """The speculative-sync chain kernel's byte-permute composition of slot
    maps (slot_compose, hjd_entropy.hpp) equals the bytewise definition."""
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "slot_compose")
        src = os.path.join(REPO, "tools", "check", "slot_compose.hip")
        inc = [f"-I{os.path.join(REPO, 'ocljpegdecoder_amd', 'csrc')}", f"-I{os.path.join(REPO, 'include')}"]
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", *inc, src, "-o", exe],
                       check=True, capture_output=True, timeout=300)
        p = subprocess.run([exe, "100000"], capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stdout + p.stderr
        assert "mismatches 0" in p.stdout
