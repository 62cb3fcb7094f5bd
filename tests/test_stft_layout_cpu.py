"""The lane-exchange FFT of `stft_mel0_kernel` (features.hip) restated in numpy: data layout and index algebra.

The kernel holds a 1024-point complex frame as 16 registers x 64 lanes (z[lane + 64 r]), runs a radix-16 DFT over
the registers, the four-step twiddles W1024^{lane k1}, then six radix-2 decimation-in-frequency stages over the lane
index, each of which first SWAPS the lane bit it works on with a register bit (lane_swap<J>: x'[l] = l_J ? y[l - 2^J]
: x[l], y'[l] = l_J ? y[l] : x[l + 2^J]) so that both butterfly inputs sit in one lane.  Afterwards register r of
lane l holds X[bin_lane(l) + 64 bin_reg(r)]; the real-FFT split takes the conjugate partner N - f from lane
lane_of_bin(64 - fl), register r ^ 15 (lane 0: its own register for (16 - m) mod 16).  This test runs exactly that
sequence of exchanges on numpy arrays and checks the bins against numpy's FFT, so the index algebra the kernel
encodes is pinned independently of the GPU (the GPU kernel itself is checked against the mel oracle in
test_features_gpu.py).  The hardware semantics of each exchange primitive were checked on the box with
scripts/probe/lane_probe.hip."""
import numpy as np


def W(n, N):
    return np.exp(-2j * np.pi * n / N)


def bin_reg(r):
    return ((r >> 1) & 1) | (r & 1) << 1 | ((r >> 3) & 1) << 2 | ((r >> 2) & 1) << 3


def bin_lane(l):
    return (l >> 2) | ((l >> 1) & 1) << 4 | (l & 1) << 5


def lane_of_bin(g):
    return ((g & 15) << 2) | ((g >> 4) & 1) << 1 | ((g >> 5) & 1)


def lane_swap(x, y, J):
    d = 1 << J
    lanes = np.arange(64)
    hi = (lanes & d) != 0
    nx, ny = x.copy(), y.copy()
    nx[hi] = y[lanes[hi] - d]
    ny[~hi] = x[lanes[~hi] + d]
    return nx, ny


def lane_fft(z):
    """registers [16][64] after the kernel's radix-16, twiddle and six lane stages"""
    a = z.reshape(16, 64)                              # a[r][l] = z[l + 64 r]
    k1 = np.arange(16)[:, None]
    r = np.arange(16)[None, :]
    Y = (W(k1 * r, 16) @ a)                            # radix 16 over the registers
    v = Y * W(np.arange(64)[None, :] * k1, 1024)       # four-step twiddles
    lanes = np.arange(64)
    for J, RB in [(5, 3), (4, 2), (3, 1), (2, 0), (1, 3), (0, 2)]:
        tw = W((lanes & ((1 << J) - 1)) << (5 - J), 64)
        for q in range(16):
            if q & (1 << RB):
                continue
            x, y = lane_swap(v[q], v[q | (1 << RB)], J)
            v[q], v[q | (1 << RB)] = x + y, (x - y) if J == 0 else (x - y) * tw
    return v


def test_lane_fft_layout_matches_numpy():
    rng = np.random.default_rng(0)
    z = rng.standard_normal(1024) + 1j * rng.standard_normal(1024)
    v = lane_fft(z)
    X = np.fft.fft(z)
    got = np.array([[v[r][l] for l in range(64)] for r in range(16)])
    want = np.array([[X[bin_lane(l) + 64 * bin_reg(r)] for l in range(64)] for r in range(16)])
    assert np.abs(got - want).max() < 1e-9 * np.abs(X).max()
    # the layout covers every bin exactly once
    bins = sorted(bin_lane(l) + 64 * bin_reg(r) for l in range(64) for r in range(16))
    assert bins == list(range(1024))


def test_real_split_with_partner_exchange_matches_rfft():
    rng = np.random.default_rng(1)
    x = rng.standard_normal(2048)
    v = lane_fft(x[0::2] + 1j * x[1::2])
    P = np.zeros(1025)
    for l in range(64):
        fl = bin_lane(l)
        pl = lane_of_bin((64 - fl) & 63)
        for r in range(16):
            m = bin_reg(r)
            zf = v[r][l]
            zc = v[r ^ 15][pl] if l else v[bin_reg((16 - m) & 15)][l]
            w = W(fl + 64 * m, 2048)
            ex, ey = zf.real + zc.real, zf.imag - zc.imag
            ox, oy = zf.imag + zc.imag, zc.real - zf.real
            re = ox * w.real - oy * w.imag + ex
            im = ox * w.imag + oy * w.real + ey
            P[fl + 64 * m] = 0.25 * (re * re + im * im)
    P[1024] = (v[0][0].real - v[0][0].imag) ** 2       # Nyquist from lane 0, register 0 (Z[0])
    ref = np.abs(np.fft.rfft(x)) ** 2
    assert np.abs(P - ref).max() < 1e-9 * ref.max()
