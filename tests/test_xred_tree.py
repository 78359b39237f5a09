"""CPU model of the multi-token engine's transposed row totals (llm_prefill.hip stream_rows_bx /
xreduce) against the decode's row_total (llm_device.h sum8_f + sum_lanes7), lane by lane in
float32: the reduce-scatter must give every total bit for bit, for Q8_0 (tree over lane bits
0..5) and for K-quants (bits 3..5 over lanes 8k+7), for the group shapes the kernels use."""
import numpy as np
import pytest

f32 = np.float32


def decode_row_total(v, kquant):
    """sum8_f (row_shr 1/2/4 prefix: lane i += lane i-1, i-2, i-4 within 16-lane rows, zero
    past the row start) then sum_lanes7 (row_shr 8, row_bcast 15 / 31), read at lane 63.
    K-quants skip sum8_f (their 8-lane sums are exact integers, valid in lanes 8k+7)."""
    v = v.astype(f32).copy()

    def shr(x, n):  # DPP row_shr:n, bound_ctrl off, old = 0
        out = np.zeros_like(x)
        for i in range(64):
            if (i % 16) >= n:
                out[i] = x[i - n]
        return out

    if not kquant:
        for n in (1, 2, 4):
            v = (v + shr(v, n)).astype(f32)
    v = (v + shr(v, 8)).astype(f32)
    b = np.zeros_like(v)  # row_bcast15, row mask 0xA: rows 1, 3 get lane 15 of the row before
    for i in range(64):
        if (i // 16) in (1, 3):
            b[i] = v[(i // 16) * 16 - 1]
    v = (v + b).astype(f32)
    b = np.zeros_like(v)  # row_bcast31, row mask 0xC: rows 2, 3 get lane 31
    for i in range(64):
        if (i // 16) in (2, 3):
            b[i] = v[31]
    v = (v + b).astype(f32)
    return v[63]


def xreduce(vals, lb, nf):
    """vals[lane][j] (64 x N): levels lb..5, scatter while a lane holds more than nf values,
    then all-reduce; returns per lane its remaining values (64 x max(nf, N >> (6 - lb)))."""
    v = [list(map(f32, vals[l])) for l in range(64)]
    n = len(v[0])
    for b in range(lb, 6):
        if n > nf:
            h = n // 2
            nv = []
            for l in range(64):
                p = l ^ (1 << b)
                if (l >> b) & 1:
                    nv.append([f32(v[l][i + h] + v[p][i + h]) for i in range(h)])
                else:
                    nv.append([f32(v[l][i] + v[p][i]) for i in range(h)])
            v, n = nv, h
        else:
            v = [[f32(v[l][i] + v[l ^ (1 << b)][i]) for i in range(n)] for l in range(64)]
    return v


@pytest.mark.parametrize("tb,ru,nm,kquant", [(8, 1, 2, False), (8, 2, 1, False), (8, 1, 1, False),
                                             (8, 2, 2, False), (8, 2, 2, True), (8, 1, 2, True),
                                             (4, 1, 2, True), (8, 1, 1, True)])
def test_reduce_scatter_equals_decode_tree(tb, ru, nm, kquant):
    rng = np.random.default_rng(tb * 100 + ru * 10 + nm + kquant)
    n = tb * ru * nm
    lb = 3 if kquant else 0
    nf = max(n >> (6 - lb), nm)
    sl = int(np.log2(n // nf))
    for trial in range(3):
        # wide dynamic range so any change of association shows in the low bits
        vals = (rng.standard_normal((64, n)) * np.exp(rng.uniform(-8, 8, (64, n)))).astype(f32)
        if kquant:  # only lanes 8k+7 carry values (sum8_i left partial sums elsewhere)
            vals[[l for l in range(64) if l % 8 != 7]] = rng.standard_normal((56, n)).astype(f32) * 1e6
        want = [decode_row_total(vals[:, j], kquant) for j in range(n)]
        got = xreduce(vals, lb, nf)
        seen = set()
        for lane in range(64):
            if kquant and lane % 8 != 7:
                continue
            if (lane >> (lb + sl)) != 0:
                continue
            jb = sum(((lane >> (lb + k)) & 1) * (n >> (k + 1)) for k in range(sl))
            for i in range(len(got[lane])):
                j = jb + i
                assert got[lane][i].tobytes() == want[j].tobytes(), (lane, j, got[lane][i], want[j])
                seen.add(j)
        assert seen == set(range(n))
