"""The two-pass batch drawing of the hybrid case (madpose_amd/csrc/host/batch_draw.h)
against the draw-by-draw loop (IterationStream::next, the reference's per-iteration
SelectMinimalSolver + HybridUniformSampling, src/hybrid_ransac.h:210-243): identical
solver types, iteration lists, kept sample indices, snapshots and stream end states,
including tiny n (duplicates and Lemire rejections take the slow path), the sf / tf
sample sizes, single-iteration batches and a one-solver prior; the scalar passes and the
AVX-512 ones (batch_draw_simd.h, with the AVX-512 MT19937 twist of rng.h).  Host
compiler only."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
HOST = os.path.join(os.path.dirname(HERE), "madpose_amd", "csrc", "host")


def test_two_pass_batch_drawing_matches_draw_by_draw(tmp_path):
    exe = str(tmp_path / "sampler_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-march=x86-64-v3", "-I", HOST,
                    os.path.join(HERE, "sampler_check.cpp"), "-o", exe], check=True)
    # mode 1: the scalar two passes; mode 2: on AVX-512 (batch_draw_simd.h), skipped on
    # a host without it
    for mode in ("1", "2"):
        r = subprocess.run([exe, mode], capture_output=True, text=True, timeout=120)
        print(r.stdout)
        assert r.returncode == 0 and (r.stdout.startswith("OK") or r.stdout.startswith("SKIP")), r.stdout + r.stderr
