"""CPU check of the sensor kernel's ray end-point arithmetic (nascargymnasium_amd/csrc/nascar_rays.h):
the header is compiled for the host with g++ and every ray's f32 end point is compared with the direct
Python-float evaluation of src/distance_sensor.py:95-103 (glibc sincos of sa) on random car poses."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ray_end_points_match_direct_evaluation(tmp_path):
    exe = tmp_path / "rays_harness"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "rays_harness.cpp")], check=True)
    out = subprocess.run([str(exe), "300000"], capture_output=True, text=True, check=True).stdout.split()
    cases, bad, fallbacks = map(int, out)
    assert cases == 300000 * 16
    assert bad == 0
    assert fallbacks < cases // 1000   # the direct-sincos fallback is rare (exact-angle ties only)


def test_glibc_sincosf_restatement_matches_host_libm(tmp_path):
    """nascar_math.h glibc_sincosf (b2Rot::Set's sinf/cosf on the device: load-free, and since round 5 one
    straight-line path with both polynomials side by side) equals the host glibc on every 61st float bit pattern.
    NASCAR_SINCOS_STRIDE=1 reruns it over all 2^32 bit patterns (the whole float range, ~1-2 min on 8 threads; run
    that way in round 5: 0 mismatches)."""
    stride = int(os.environ.get("NASCAR_SINCOS_STRIDE", "61"))
    exe = tmp_path / "sincosf_harness"
    subprocess.run(["hipcc", "-O2", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "sincosf_harness.cpp")], check=True)
    checked, bad = map(int, subprocess.run([str(exe), str(stride), "8"], capture_output=True, text=True,
                                           check=True).stdout.split())
    assert checked >= 0.99 * (1 << 32) / stride and bad == 0     # (the finite floats: 99.6 % of the patterns)
