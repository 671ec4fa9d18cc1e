"""Host-side checks of the two-pass FFT plan (csrc/hip/fft_two_pass.hip,
opt-in BRP_TWO_PASS=1): its index algebra -- pass A's output positions are a
permutation of a column and the inverse of tp_pos, the swizzled LDS block and
the Stockham stages cover every element once, pass B's row tiles stay inside a
column (hipk::two_pass_selftest, shared helpers with the kernel)."""


def test_two_pass_index_algebra(brp):
    assert brp.two_pass_selftest() == ""
