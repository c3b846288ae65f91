"""Generator bit-exactness vs libstdc++ (the reference's std::mt19937 +
uniform_real_distribution<float>(-100,100), Utility.cpp:6-18) including jump-ahead slices
(kdtree_mpi.cpp:19-41)."""
import subprocess

import numpy as np
import pytest
import torch

import parallel_kd_tree_amd as pk

GOLDEN = r"""
#include <random>
#include <cstdio>
#include <cstdlib>
int main(int argc, char** argv) {
  int seed = atoi(argv[1]); long long skip = atoll(argv[2]); long long cnt = atoll(argv[3]);
  std::mt19937 r(seed); std::uniform_real_distribution<float> d(-100, 100);
  for (long long i = 0; i < skip; ++i) d(r);
  for (long long i = 0; i < cnt; ++i) { float v = d(r); fwrite(&v, 4, 1, stdout); }
}
"""


@pytest.fixture(scope="module")
def golden(tmp_path_factory):
    d = tmp_path_factory.mktemp("golden")
    src = d / "g.cpp"
    src.write_text(GOLDEN)
    exe = d / "g"
    subprocess.run(["g++", "-O2", "-std=c++17", str(src), "-o", str(exe)], check=True)

    def run(seed, skip, cnt):
        out = subprocess.run([str(exe), str(seed), str(skip), str(cnt)], check=True, capture_output=True).stdout
        return np.frombuffer(out, dtype=np.float32)
    return run


@pytest.mark.parametrize("seed,dim,n", [(42, 3, 1034), (0, 128, 50), (7, 1, 5000), (123456, 8, 777)])
def test_problem_matches_libstdcxx(golden, seed, dim, n):
    x = pk.generate_problem(seed, dim, n)
    assert x.shape == (n, dim) and x.dtype == torch.float32
    np.testing.assert_array_equal(x.numpy().ravel(), golden(seed, 0, n * dim))


@pytest.mark.parametrize("first,rows,dim", [(1, 10, 3), (333, 50, 3), (100000, 64, 3), (4_000_000, 16, 3),
                                             (1234, 20, 128)])
def test_slice_jump_ahead(golden, first, rows, dim):
    x = pk.generate_slice(5, dim, first, rows)
    np.testing.assert_array_equal(x.numpy().ravel(), golden(5, first * dim, rows * dim))


def test_threaded_slice_equals_serial():
    a = pk.generate_slice(9, 3, 12345, 3_000_000, threads=8)
    b = pk.generate_slice(9, 3, 12345, 3_000_000, threads=1)
    assert torch.equal(a, b)


def test_uniform_value_map():
    from parallel_kd_tree_amd.utils.generator import u32_to_uniform
    u = torch.tensor([0, 1, 2**31, 2**32 - 1, 2**32 - 128], dtype=torch.int64)
    v = u32_to_uniform(u)
    assert v[0] == -100.0 and v.max() < 100.0 and v.min() >= -100.0


@pytest.mark.parametrize("seed,first,rows,dim", [(5, 0, 10, 3), (5, 17, 40_000, 3), (42, 1, 333_333, 1),
                                                  (3, 99_991, 100_000, 3), (11, 0, 7_000, 128)])
def test_device_algorithm_emulated(seed, first, rows, dim):
    """The device generator's chunk plan and jump rounds, run on the host, equal the stream."""
    from parallel_kd_tree_amd.utils.generator import generate_emulated
    from parallel_kd_tree_amd.ops import native
    S, C, R = native().devgen_plan(rows * dim)
    assert C * S >= rows * dim and (1 << R) >= C
    assert torch.equal(generate_emulated(seed, dim, first, rows), pk.generate_slice(seed, dim, first, rows))


@pytest.mark.gpu
@pytest.mark.parametrize("seed,first,rows,dim", [(5, 0, 10, 3), (5, 17, 40_000, 3), (42, 1, 333_333, 1),
                                                  (3, 12_500_000, 2_000_000, 3), (11, 0, 7_000, 128),
                                                  (42, 0, 25_000_000, 3)])
def test_device_generator_bit_exact(seed, first, rows, dim):
    x = pk.generate_slice(seed, dim, first, rows, device="cuda")
    torch.cuda.synchronize()
    assert x.is_cuda and x.shape == (rows, dim)
    assert torch.equal(x.cpu(), pk.generate_slice(seed, dim, first, rows))
