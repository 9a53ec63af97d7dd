"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, the
reference-generated golden fixtures, and size-independent properties at the
BASELINE.json shapes.  Bit-exact everywhere (integer/byte work)."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def dev_tensor(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def gpu_encode(leo, data: np.ndarray, r: int) -> np.ndarray:
    out = leo.encode(dev_tensor(data), r)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def gpu_decode(leo, data, recovery, lost_o, lost_r):
    res = leo.decode(dev_tensor(data), dev_tensor(recovery), lost_o, lost_r)
    torch.cuda.synchronize()
    return {i: v.cpu().numpy() for i, v in res.items()}


# ---------------------------------------------------------------- encode --

ENC_CASES = [
    (2, 2, 64), (3, 2, 64), (4, 4, 128), (7, 5, 128), (16, 16, 64), (17, 16, 192), (32, 32, 256),
    (33, 9, 64), (64, 64, 320), (100, 20, 64), (128, 128, 128), (130, 126, 64), (200, 55, 64), (250, 6, 64),
    (5, 3, 64 * 17), (64, 64, 64 * 33),  # column tails that are not a whole tile
    # FF16 single-tile encoders (m <= 256) and multi-pass ones (m > 256)
    (129, 127, 64), (300, 37, 128), (1000, 200, 64), (700, 256, 128), (600, 300, 64), (5000, 3000, 64),
    (2000, 1000, 128),
    # narrow-strip encoder: m = 128 on 32-unit strips (60-64 KiB pieces), full strips and a
    # last strip of 8 units (61504 B = 240 strips of 32 units + 8); m = 256 on 16-unit strips
    (200, 100, 65536), (300, 100, 61504), (1000, 200, 61504),
]


@pytest.mark.parametrize("k,r,b", ENC_CASES)
def test_encode_matches_oracle(leo, k, r, b):
    rng = np.random.default_rng(k * 7919 + r * 31 + b)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    expect = ol.oracle().encode(data, r)
    got = gpu_encode(leo, data, r)
    assert np.array_equal(got, expect)


def _golden_small():
    return np.load(os.path.join(GOLDEN, "golden_small.npz"))


def _golden_keys(prefix):
    with np.load(os.path.join(GOLDEN, "golden_small.npz")) as z:
        return sorted(k for k in z.files if k.startswith(prefix))


@pytest.mark.parametrize("key", _golden_keys("enc_"))
def test_encode_matches_reference_golden(leo, key):
    k, r, b = (int(x) for x in key.split("_")[1:])
    with _golden_small() as z:
        expect = z[key]
    data = ol.pcg_bytes(2, 0, k, b)
    got = gpu_encode(leo, data, r)
    assert np.array_equal(got, expect)


def test_encode_host_memory_matches_oracle(leo):
    """Reference contract: caller-owned host buffers in and out (leopard.h:147-186)."""
    for (k, r, b) in [(128, 128, 1024), (1000, 200, 256), (3, 2, 64)]:
        rng = np.random.default_rng(k + r)
        data = rng.integers(0, 256, (k, b), dtype=np.uint8)
        wc = leo.leo_encode_work_count(k, r)
        work = np.zeros((wc, b), dtype=np.uint8)
        res = leo.leo_encode(b, k, r, wc, [data[i].ctypes.data for i in range(k)],
                             [work[i].ctypes.data for i in range(wc)])
        assert res == leo.LeopardResult.Success, leo.last_error()
        assert np.array_equal(work[:r], ol.oracle().encode(data, r))


# ---------------------------------------------------------------- decode --

DEC_CASES = [  # (K, R, B, originals lost)
    (2, 2, 64, 1), (3, 2, 64, 2), (7, 5, 128, 5), (16, 16, 64, 9), (100, 20, 64, 20), (128, 128, 128, 128),
    (128, 128, 64, 1), (130, 126, 64, 100), (200, 55, 64, 55), (64, 64, 64 * 33, 40),
    (129, 127, 64, 127), (300, 37, 128, 30),
    # every original lost (K = R, the half-position decoder), R not a power of 2
    (90, 90, 64 * 5, 90), (3, 3, 64, 3), (33, 33, 256, 33),
    (300, 300, 128, 300), (600, 600, 64, 600), (2000, 2000, 64, 2000),  # FF16 half-position pass 2
    (1000, 200, 64, 200), (600, 300, 64, 299), (5000, 3000, 64, 3000),
    # every original lost with K = R = m: the inverse-transform decoder (launch_ff8_decode_full),
    # single tile (64 KiB-piece form) and the wide form (>= 256 KiB pieces)
    (2, 2, 64, 2), (4, 4, 64 * 3, 4), (16, 16, 64 * 33, 16), (64, 64, 256, 64), (128, 128, 1 << 18, 128),
    # some originals received with n = 2m: the split decoder (k_ff8_dec_split), K <= m
    (128, 128, 65536, 16), (60, 40, 64 * 5, 30), (8, 5, 64, 3), (128, 128, 1 << 18, 127), (32, 32, 64, 31),
]


@pytest.mark.parametrize("k,r,b,loss", DEC_CASES)
def test_decode_roundtrip_and_oracle(leo, k, r, b, loss):
    rng = np.random.default_rng(k * 13 + r + loss)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    rec = ol.oracle().encode(data, r)
    lost_o = sorted(rng.choice(k, loss, replace=False).tolist())
    lost_r = sorted(rng.choice(r, r - loss, replace=False).tolist())
    got = gpu_decode(leo, data, rec, lost_o, lost_r)
    for i in lost_o:
        assert np.array_equal(got[i], data[i]), i
    # non-codeword input: the exact decoder map must equal the oracle's
    junk = rng.integers(0, 256, (r, b), dtype=np.uint8)
    expect = ol.oracle().decode(data, junk, lost_o, lost_r)
    got = gpu_decode(leo, data, junk, lost_o, lost_r)
    for i in lost_o:
        assert np.array_equal(got[i], expect[i]), i


# The GF(2^8) matrix path (rs_ff8_mat.hip, leopard_amd.cpp use_matrix): small codes and few
# losses run as the L x N coefficient matrix built from the transform kernels' outputs on
# unit pieces.  Shapes on it (the breadth lines 100+10 / 100+20, the 16-loss headline shape,
# output groups of 4 and 8, lost recovery pieces), each encode and decode repeated so
# the second call reads the cached matrix.
MAT_CASES = [(100, 10, 2560, 10, 0), (100, 20, 2560, 20, 0), (128, 128, 65536, 16, 0), (64, 32, 4096, 16, 5),
             (32, 8, 65536, 4, 2), (16, 16, 64, 1, 3), (200, 30, 256, 29, 0), (7, 5, 64 * 9, 3, 1),
             # round 6 (decodes up to L N B = 2^29; output groups of 8; up to 256 inputs)
             (128, 128, 262144, 8, 120), (128, 128, 65536, 32, 0), (100, 10, 65536, 10, 0), (12, 3, 64 * 1000, 1, 0),
             (100, 4, 262144, 4, 0)]  # 4-dword lanes (L <= 4 on many strips)


@pytest.mark.parametrize("k,r,b,loss,rec_lost", MAT_CASES)
def test_matrix_path_matches_oracle(leo, k, r, b, loss, rec_lost):
    rng = np.random.default_rng(k * 5 + r * 3 + b + loss)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    expect = ol.oracle().encode(data, r)
    for _ in range(2):
        assert np.array_equal(gpu_encode(leo, data, r), expect)
    lost_o = sorted(rng.choice(k, loss, replace=False).tolist())
    # r - loss recovery pieces are needed at least; rec_lost of the others are missing too
    lost_r = sorted(rng.choice(r, min(rec_lost, r - loss), replace=False).tolist())
    for _ in range(2):
        got = gpu_decode(leo, data, expect, lost_o, lost_r)
        for i in lost_o:
            assert np.array_equal(got[i], data[i]), i
    junk = rng.integers(0, 256, (r, b), dtype=np.uint8)  # not a codeword: the exact decoder map
    want = ol.oracle().decode(data, junk, lost_o, lost_r)
    got = gpu_decode(leo, data, junk, lost_o, lost_r)
    for i in lost_o:
        assert np.array_equal(got[i], want[i]), i


def test_matrix_built_on_one_stream_used_on_another(leo):
    """A matrix generated by a call on stream A and used at once by an async call
    on stream B (B waits for A's generation on the device, no host sync)."""
    k, r, b, loss = 90, 17, 4096, 11
    rng = np.random.default_rng(17)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    rec = ol.oracle().encode(data, r)
    lost_o = sorted(rng.choice(k, loss, replace=False).tolist())
    lost_r = sorted(rng.choice(r, 2, replace=False).tolist())
    orig, recd = dev_tensor(data), dev_tensor(rec)
    torch.cuda.synchronize()
    outs = []
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    leo.set_async(True)
    try:
        for st in (sa, sb):
            leo.set_stream(st.cuda_stream)
            with torch.cuda.stream(st):
                outs.append(leo.decode(orig, recd, lost_o, lost_r))
    finally:
        leo.set_async(False)
        leo.set_stream(None)
    torch.cuda.synchronize()
    for o in outs:
        for i in lost_o:
            assert np.array_equal(o[i].cpu().numpy(), data[i]), i


_TRANSFORM_ONLY = r"""
import sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, {tests!r})
import leopard_amd as leo, test_gpu_parity as t
assert leo.leo_init() == 0
n = 0
for k, r, b in t.ENC_CASES:
    if k + r <= 256:
        t.test_encode_matches_oracle(leo, k, r, b); n += 1
for k, r, b, loss in t.DEC_CASES:
    if k + r <= 256:
        t.test_decode_roundtrip_and_oracle(leo, k, r, b, loss); n += 1
for c in t.MAT_CASES:
    t.test_matrix_path_matches_oracle(leo, *c); n += 1
print("transform ok", n)
"""


def test_ff8_transform_kernels_with_matrix_path_off():
    """The GF(2^8) shapes of ENC_CASES / DEC_CASES / MAT_CASES through the transform
    kernels alone (experiment build, LEO_AMD_FF8_MATRIX=0), in a child process:
    the product routes many of them to the matrix path, which is built from
    these kernels."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    lib = os.path.join(repo, "leopard_amd", "lib", "exp", "libleopard_amd.so")
    env = dict(os.environ, LEOPARD_AMD_LIB=lib, LEO_AMD_FF8_MATRIX="0")
    p = subprocess.run([sys.executable, "-c", _TRANSFORM_ONLY.format(repo=repo, tests=here)], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0 and "transform ok" in p.stdout, (p.stdout[-2000:], p.stderr[-3000:])


# The single-pass GF(2^16) decoder (k_dec16n_one: n <= 2048, <= 4 tiles of originals,
# pieces >= 60 KiB): a tile mixing recovery and original positions (m = 128), a last
# column strip of 8 units (B = 64 mod 128) in the 16-unit form and of one 64-byte
# block in the 32-unit form (60-64 KiB pieces), lost recovery pieces, every
# original lost, and callers' pointer tables (pieces scattered over a store's rows).
@pytest.mark.parametrize("k,r,b,loss,layout", [(300, 100, 65600, 60, "slab"), (1000, 200, 61504, 150, "scattered"),
                                               (500, 500, 65536, 500, "slab"), (1000, 200, 81984, 180, "slab"),
                                               (600, 400, 65536, 300, "scattered")])
def test_single_pass_ff16_decoder_matches_oracle(leo, k, r, b, loss, layout):
    rng = np.random.default_rng(k + r + loss)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    junk = rng.integers(0, 256, (r, b), dtype=np.uint8)  # not a codeword: the exact decoder map is compared
    lost_o = sorted(rng.choice(k, loss, replace=False).tolist())
    lost_r = sorted(rng.choice(r, r - loss, replace=False).tolist())
    expect = ol.oracle().decode(data, junk, lost_o, lost_r)
    wc = leo.leo_decode_work_count(k, r)
    if layout == "slab":
        orig, rec = dev_tensor(data), dev_tensor(junk)
        work = torch.zeros((wc, b), dtype=torch.uint8, device="cuda")
        po = [orig[i].data_ptr() for i in range(k)]
        pr = [rec[i].data_ptr() for i in range(r)]
        pw = [work[i].data_ptr() for i in range(wc)]
        row = {i: i for i in range(wc)}
    else:
        perm_o, perm_r, perm_w = rng.permutation(k), rng.permutation(r), rng.permutation(wc)
        orig = dev_tensor(data[np.argsort(perm_o)])  # piece i at row perm_o[i]
        rec = dev_tensor(junk[np.argsort(perm_r)])
        work = torch.zeros((wc, b), dtype=torch.uint8, device="cuda")
        po = [orig[int(perm_o[i])].data_ptr() for i in range(k)]
        pr = [rec[int(perm_r[i])].data_ptr() for i in range(r)]
        pw = [work[int(perm_w[i])].data_ptr() for i in range(wc)]
        row = {i: int(perm_w[i]) for i in range(wc)}
    lo, lr = set(lost_o), set(lost_r)
    res = leo.leo_decode(b, k, r, wc, [None if i in lo else po[i] for i in range(k)],
                         [None if i in lr else pr[i] for i in range(r)], pw)
    assert res == leo.LeopardResult.Success, leo.last_error()
    torch.cuda.synchronize()
    got = work.cpu().numpy()
    for i in lost_o:
        assert np.array_equal(got[row[i]], expect[i]), i


@pytest.mark.parametrize("key", _golden_keys("decout_"))
def test_decode_matches_reference_golden(leo, key):
    k, r, b, loss = (int(x) for x in key.split("_")[1:])
    tag = "_".join(key.split("_")[1:])
    with _golden_small() as z:
        lo = z["declo_" + tag].tolist()
        lr = z["declr_" + tag].tolist()
        expect = z[key]
    data = ol.pcg_bytes(2, 1, k, b)
    rec = ol.pcg_bytes(2, 2, r, b)
    got = gpu_decode(leo, data, rec, lo, lr)
    for j, i in enumerate(lo):
        assert np.array_equal(got[i], expect[j]), i


def test_decode_benchmark_loss_pattern(leo):
    """tests/benchmark.cpp:440-467 loss pattern with its self-checking packets."""
    k, r, b = 1000, 200, 640
    data = ol.pcg_bytes(2, 0, k, b)
    rec = gpu_encode(leo, data, r)
    lo, lr = ol.benchmark_losses(k, r, r, seed=2, trial=0, data_bytes=k * b)
    got = gpu_decode(leo, data, rec, lo, lr)
    for i in lo:
        assert np.array_equal(got[i], data[i])


def test_decode_host_memory(leo):
    k, r, b = 128, 128, 512
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    rec = ol.oracle().encode(data, r)
    lost = list(range(0, k, 2))
    lost_r = list(range(len(lost), r))
    wc = leo.leo_decode_work_count(k, r)
    work = np.zeros((wc, b), dtype=np.uint8)
    res = leo.leo_decode(b, k, r, wc, [None if i in lost else data[i].ctypes.data for i in range(k)],
                         [None if i in lost_r else rec[i].ctypes.data for i in range(r)],
                         [work[i].ctypes.data for i in range(wc)])
    assert res == leo.LeopardResult.Success, leo.last_error()
    for i in lost:
        assert np.array_equal(work[i], data[i])


# ------------------------------------------------------------ edge paths --

def test_edge_paths(leo):
    rng = np.random.default_rng(9)
    # K == 1 (leopard.cpp:144-149, 279-283)
    d = rng.integers(0, 256, (1, 128), dtype=np.uint8)
    assert np.array_equal(gpu_encode(leo, d, 1), d)
    # R == 1 parity (leopard.cpp:106-121, 214-231)
    d = rng.integers(0, 256, (9, 192), dtype=np.uint8)
    par = gpu_encode(leo, d, 1)
    assert np.array_equal(par[0], np.bitwise_xor.reduce(d, axis=0))
    got = gpu_decode(leo, d, par, [4], [])
    assert np.array_equal(got[4], d[4])
    # zero loss: every original copied to work (leopard.cpp:286-291)
    d = rng.integers(0, 256, (20, 64), dtype=np.uint8)
    rec = gpu_encode(leo, d, 5)
    k, r = 20, 5
    work = torch.zeros((leo.leo_decode_work_count(k, r), 64), dtype=torch.uint8, device="cuda")
    dt, rt = dev_tensor(d), dev_tensor(rec)
    res = leo.leo_decode(64, k, r, work.shape[0], [dt[i].data_ptr() for i in range(k)],
                         [rt[i].data_ptr() for i in range(r)], [work[i].data_ptr() for i in range(work.shape[0])])
    assert res == leo.LeopardResult.Success
    assert np.array_equal(work[:k].cpu().numpy(), d)


def test_error_codes(leo):
    R = leo.LeopardResult
    t = torch.zeros((8, 64), dtype=torch.uint8, device="cuda")
    p = [t[i].data_ptr() for i in range(8)]
    assert leo.leo_encode(63, 4, 2, 4, p[:4], p[4:]) == R.InvalidSize
    assert leo.leo_encode(0, 4, 2, 4, p[:4], p[4:]) == R.InvalidSize
    assert leo.leo_encode(64, 4, 5, 4, p[:4], p[4:]) == R.InvalidCounts
    assert leo.leo_encode(64, 4, 0, 4, p[:4], p[4:]) == R.InvalidCounts
    assert leo.leo_encode(64, 4, 2, 3, p[:4], p[4:]) == R.InvalidCounts
    assert leo.leo_encode(64, 4, 2, 4, None, p[4:]) == R.InvalidInput
    assert leo.leo_decode(64, 4, 2, 8, [None, None, None, p[3]], [p[4], p[5]], p) == R.NeedMoreData
    assert leo.leo_decode(64, 4, 2, 7, [None, p[1], p[2], p[3]], [p[4], p[5]], p) == R.InvalidCounts
    # n = NextPow2(NextPow2(R) + K) > 65536
    assert leo.leo_encode_work_count(60000, 10000) == 32768
    big = [p[0]] * 60000
    assert leo.leo_encode(64, 60000, 10000, 32768, big, [p[1]] * 32768) == R.TooMuchData


def test_slice_api_matches_whole(leo):
    """Column sharding primitive: encoding byte ranges separately == whole."""
    k, r, b = 100, 30, 64 * 40
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    expect = ol.oracle().encode(data, r)
    dt = dev_tensor(data)
    wc = leo.leo_encode_work_count(k, r)
    work = torch.zeros((wc, b), dtype=torch.uint8, device="cuda")
    for lo in range(0, b, 64 * 10):
        res = leo.leo_amd_encode_slice(b, lo, 64 * 10, k, r, wc, [dt[i].data_ptr() for i in range(k)],
                                       [work[i].data_ptr() for i in range(wc)])
        assert res == leo.LeopardResult.Success
    torch.cuda.synchronize()
    assert np.array_equal(work[:r].cpu().numpy(), expect)


def test_scattered_pointer_tables(leo):
    """Non-slab piece arrays exercise the uploaded pointer-table path."""
    k, r, b = 50, 20, 256
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    perm = rng.permutation(k)
    store = dev_tensor(data[perm])  # piece i lives at row inv[i]
    inv = np.argsort(perm)
    wc = leo.leo_encode_work_count(k, r)
    work = torch.zeros((wc, b), dtype=torch.uint8, device="cuda")
    wperm = rng.permutation(wc)
    res = leo.leo_encode(b, k, r, wc, [store[int(inv[i])].data_ptr() for i in range(k)],
                         [work[int(wperm[i])].data_ptr() for i in range(wc)])
    assert res == leo.LeopardResult.Success
    torch.cuda.synchronize()
    got = work.cpu().numpy()[wperm[:r]]
    assert np.array_equal(got, ol.oracle().encode(data, r))


# ----------------------------------------------- BASELINE shapes (full size) --

def _digests(kind="hash_digests"):
    path = os.path.join(GOLDEN, "golden_digests.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f).get(kind, {})


def _sha_rows(t, rows):
    """sha256 of rows of a device tensor concatenated in the given order."""
    h = hashlib.sha256()
    for i in rows:
        h.update(t[i].cpu().numpy().tobytes())
    return h.hexdigest()


BIG = [(128, 128, 65536), (128, 128, 64000), (1000, 200, 65536), (1000, 200, 64000), (32768, 32768, 65536)]


@pytest.mark.slow
@pytest.mark.parametrize("k,r,b", BIG)
def test_baseline_shapes_digest_and_roundtrip(leo, k, r, b):
    key = f"{k}_{r}_{b}"
    dig = _digests().get(key)
    data = ol.hash_bytes_torch(7, k, b, "cuda")
    rec = leo.encode(data, r)
    torch.cuda.synchronize()
    if dig is not None:
        h = hashlib.sha256(rec.contiguous().cpu().numpy().tobytes()).hexdigest()
        assert h == dig, "recovery bytes differ from the reference library's"
    # worst case of the BASELINE configs: lose min(R, K) originals, benchmark pattern
    lo, lr = ol.benchmark_losses(k, r, r, seed=2, trial=0)
    got = leo.decode(data, rec, lo, lr)
    torch.cuda.synchronize()
    idx = torch.tensor(lo, device="cuda")
    stacked = torch.stack([got[i] for i in lo])
    assert torch.equal(stacked, data.index_select(0, idx))
    del got, stacked
    # the decoder's exact map at full size: non-codeword "recovery" pieces,
    # digest of the rebuilt originals vs the reference library's (gen_golden.py --big-decode)
    ddig = _digests("decode_hash_digests").get(key)
    if ddig is not None:
        junk = ol.hash_bytes_torch(8, r, b, "cuda")
        work = torch.empty((leo.leo_decode_work_count(k, r), b), dtype=torch.uint8, device="cuda")
        leo.decode(data, junk, lo, lr, work=work)
        torch.cuda.synchronize()
        assert _sha_rows(work, lo) == ddig, "decoder output differs from the reference library's"


@pytest.mark.slow
def test_configs4_column_sharded_8way_digest(leo):
    """BASELINE.json configs[4]: one 32768+32768 x 64 KiB object column-sharded
    8 ways (8 KiB per piece per rank, leopard_amd.sharding over leo_amd_*_slice),
    every rank's slice run here in turn on one device.  The union must carry the
    reference library's recovery digest, rebuild every original after full loss,
    and reproduce the reference decoder's digest on non-codeword input
    (LeopardFF16.cpp:1397-1467, 1652-1775 are the codec being sharded)."""
    from leopard_amd.sharding import decode_shard, encode_shard
    k = r = 32768
    b, world = 65536, 8
    key = f"{k}_{r}_{b}"
    data = ol.hash_bytes_torch(7, k, b, "cuda")
    wc = leo.leo_encode_work_count(k, r)
    work = torch.empty((wc, b), dtype=torch.uint8, device="cuda")
    po = [data[i].data_ptr() for i in range(k)]
    pw = [work[i].data_ptr() for i in range(wc)]
    for rank in range(world):
        assert encode_shard(b, rank, world, k, r, po, pw) == 0, leo.last_error()
    torch.cuda.synchronize()
    assert _sha_rows(work, range(r)) == _digests()[key], "sharded recovery differs from the reference library's"
    dwc = leo.leo_decode_work_count(k, r)
    dwork = torch.empty((dwc, b), dtype=torch.uint8, device="cuda")
    lost = [None] * k
    pr = [work[i].data_ptr() for i in range(r)]
    pd = [dwork[i].data_ptr() for i in range(dwc)]
    for rank in range(world):
        assert decode_shard(b, rank, world, k, r, lost, pr, pd) == 0, leo.last_error()
    torch.cuda.synchronize()
    assert torch.equal(dwork[:k], data), "sharded full-loss decode did not rebuild the originals"
    del work
    junk = ol.hash_bytes_torch(8, r, b, "cuda")
    lo, lr = ol.benchmark_losses(k, r, r, seed=2, trial=0)
    los, lrs = set(lo), set(lr)
    po = [None if i in los else data[i].data_ptr() for i in range(k)]
    pr = [None if i in lrs else junk[i].data_ptr() for i in range(r)]
    for rank in range(world):
        assert decode_shard(b, rank, world, k, r, po, pr, pd) == 0, leo.last_error()
    torch.cuda.synchronize()
    assert _sha_rows(dwork, lo) == _digests("decode_hash_digests")[key], "sharded decoder map differs"


@pytest.mark.gpu
@pytest.mark.parametrize("k,r,b,world", [(128, 128, 65536, 2), (100, 60, 6400, 3), (300, 100, 64 * 37, 4)])
def test_column_shards_on_device_equal_whole_call(leo, k, r, b, world):
    """The multi-GPU path per rank: leo_amd_*_slice over this rank's column
    range (leopard_amd.sharding), run here for every rank in turn on one
    device; the union equals one whole-buffer call and the oracle."""
    import torch
    from leopard_amd.sharding import decode_shard, encode_shard
    data = ol.pcg_bytes(11, 2, k, b)
    o = torch.from_numpy(data).cuda()
    wc = leo.leo_encode_work_count(k, r)
    work = torch.zeros((wc, b), dtype=torch.uint8, device="cuda")
    for rank in range(world):
        assert encode_shard(b, rank, world, k, r, [o[i].data_ptr() for i in range(k)],
                            [work[i].data_ptr() for i in range(wc)]) == 0, leo.last_error()
    torch.cuda.synchronize()
    rec = work[:r].cpu().numpy()
    assert np.array_equal(rec, ol.oracle().encode(data, r))
    lost = list(range(0, min(k, r)))
    dwc = leo.leo_decode_work_count(k, r)
    dwork = torch.zeros((dwc, b), dtype=torch.uint8, device="cuda")
    recd = work[:r].clone()
    for rank in range(world):
        assert decode_shard(b, rank, world, k, r, [None if i in lost else o[i].data_ptr() for i in range(k)],
                            [recd[i].data_ptr() for i in range(r)],
                            [dwork[i].data_ptr() for i in range(dwc)]) == 0, leo.last_error()
    torch.cuda.synchronize()
    for i in lost:
        assert torch.equal(dwork[i], o[i]), i


# ------------------------------------------------- host-memory pipeline --

@pytest.mark.parametrize("k,r,b,loss", [(128, 128, 1 << 18, 128), (100, 30, 64 * 1000, 17), (1000, 200, 1 << 14, 200),
                                        (9, 1, 1 << 16, 1)])
def test_host_pipeline_roundtrip(leo, k, r, b, loss):
    """Host (pageable) buffers large enough to be cut into several column
    slices (two-slot ring, FF8 on two streams, FF16 on one): encode must match
    the oracle and the decode of the benchmark loss pattern must rebuild the
    originals, all in host memory (leopard.h:147-186, 205-234)."""
    data = ol.pcg_bytes(4, k, k, b)
    wc = leo.leo_encode_work_count(k, r)
    work = np.zeros((wc, b), dtype=np.uint8)
    res = leo.leo_encode(b, k, r, wc, [data[i].ctypes.data for i in range(k)], [work[i].ctypes.data for i in range(wc)])
    assert res == leo.LeopardResult.Success, leo.last_error()
    assert np.array_equal(work[:r], ol.oracle().encode(data, r))  # every slice of the pipeline
    rec = work[:r].copy()
    lo, lr = ol.benchmark_losses(k, r, loss, seed=4, trial=k)
    dwc = leo.leo_decode_work_count(k, r)
    dwork = np.zeros((dwc, b), dtype=np.uint8)
    res = leo.leo_decode(b, k, r, dwc, [None if i in lo else data[i].ctypes.data for i in range(k)],
                         [None if i in lr else rec[i].ctypes.data for i in range(r)],
                         [dwork[i].ctypes.data for i in range(dwc)])
    assert res == leo.LeopardResult.Success, leo.last_error()
    for i in lo:
        assert np.array_equal(dwork[i], data[i]), i


@pytest.mark.parametrize("k,r,b,layout", [(128, 128, 1 << 16, "strided"), (128, 128, 1 << 16, "scattered"),
                                          (1000, 200, 4096, "strided"), (1000, 200, 4096, "scattered"),
                                          (200, 55, 64 * 100, "two_arrays"), (128, 128, 1 << 16, "ascending"),
                                          (100, 20, 640, "ascending")])
def test_host_layouts_direct_and_ring(leo, k, r, b, layout):
    """The two host-memory paths: pieces forming a few row runs go by direct
    SDMA copies (1-D for dense rows, 2-D for rows of a wider array:
    "strided", "two_arrays"), pieces at scattered addresses through the
    gather / scatter ring ("scattered": one allocation per piece, handed over
    in descending address order, so no two form a run; "ascending": the same
    allocations in ascending order, where neighbours at a small gap form 2-D
    runs and larger gaps start new runs).  Encode must match the
    oracle and the decode of every lost original must rebuild it."""
    data = ol.pcg_bytes(8, k, k, b)
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)

    def rows(n, fill=None):
        if layout == "strided":  # rows of a wider array: stride b + 192
            big = np.zeros((n, b + 192), dtype=np.uint8)
            v = [big[i, 64:64 + b] for i in range(n)]
        elif layout == "two_arrays":
            h = n // 2
            a1, a2 = np.zeros((h, b), dtype=np.uint8), np.zeros((n - h, b), dtype=np.uint8)
            v = [a1[i] for i in range(h)] + [a2[i] for i in range(n - h)]
        elif layout == "ascending":  # separate allocations in ascending address order: runs only over small gaps
            v = [np.zeros(b, dtype=np.uint8) for _ in range(n)]
            v.sort(key=lambda x: x.ctypes.data)
        else:
            v = [np.zeros(b, dtype=np.uint8) for _ in range(n)]
            v.sort(key=lambda x: -x.ctypes.data)  # descending addresses: never a run
        if fill is not None:
            for i in range(n):
                v[i][:] = fill[i]
        return v

    din = rows(k, data)
    work = rows(wc)
    res = leo.leo_encode(b, k, r, wc, [x.ctypes.data for x in din], [x.ctypes.data for x in work])
    assert res == leo.LeopardResult.Success, leo.last_error()
    rec = np.stack(work[:r])
    assert np.array_equal(rec, ol.oracle().encode(data, r))
    loss = min(k, r)
    lo, lr = ol.benchmark_losses(k, r, loss, seed=8, trial=k)
    recv = rows(r, rec)
    dwork = rows(dwc)
    res = leo.leo_decode(b, k, r, dwc, [None if i in lo else din[i].ctypes.data for i in range(k)],
                         [None if i in lr else recv[i].ctypes.data for i in range(r)],
                         [x.ctypes.data for x in dwork])
    assert res == leo.LeopardResult.Success, leo.last_error()
    for i in lo:
        assert np.array_equal(dwork[i], data[i]), i


def test_host_edge_paths(leo):
    """K == 1 and zero-loss host calls are copies (leopard.cpp:143-149, 279-291)."""
    d = ol.pcg_bytes(6, 0, 1, 640)
    work = np.zeros((1, 640), dtype=np.uint8)
    assert leo.leo_encode(640, 1, 1, 1, [d[0].ctypes.data], [work[0].ctypes.data]) == 0
    assert np.array_equal(work[0], d[0])
    k, r, b = 20, 5, 192
    d = ol.pcg_bytes(6, 1, k, b)
    rec = ol.oracle().encode(d, r)
    dwc = leo.leo_decode_work_count(k, r)
    dwork = np.zeros((dwc, b), dtype=np.uint8)
    assert leo.leo_decode(b, k, r, dwc, [d[i].ctypes.data for i in range(k)], [rec[i].ctypes.data for i in range(r)],
                          [dwork[i].ctypes.data for i in range(dwc)]) == 0
    assert np.array_equal(dwork[:k], d)


@pytest.mark.gpu
@pytest.mark.parametrize("groups", [1, 2])
def test_encoder_lane_group_forms(groups):
    """The lane-group encoder forms vs the oracle.  They are A/B forms, not the
    product's: LEO_AMD_FF8_G (read once per process) selects them only in the
    experiment build of the library (lib/exp, LAMD_EXPERIMENT_ENV=1)."""
    import subprocess
    import sys
    exp = os.path.join(os.path.dirname(GOLDEN), "..", "leopard_amd", "lib", "exp", "libleopard_amd.so")
    assert os.path.exists(exp), "make -C leopard_amd builds the experiment library"
    env = dict(os.environ, LEO_AMD_FF8_G=str(groups), LEOPARD_AMD_LIB=os.path.abspath(exp))
    tool = os.path.join(os.path.dirname(GOLDEN), "..", "tools", "probe_g.py")
    res = subprocess.run([sys.executable, tool], env=env, capture_output=True, text=True, timeout=110)
    assert res.returncode == 0, res.stdout + res.stderr


# ------------------------------------------- async calls on several streams --

def test_async_calls_on_two_streams_do_not_share_scratch(leo):
    """Device-resident calls in async mode from one thread, alternating between
    two HIP streams (independent objects on different streams).
    The GF(2^16) calls keep pointer tables, the erasure state and the multi-pass
    slabs in device scratch that their kernels read after the call returns; each
    stream must get its own.  Scattered (non-slab) piece
    arrays force the pointer-table uploads; R = 1 exercises the XOR path's tables."""
    shapes = [(5000, 3000, 2048, 3000), (1000, 200, 4096, 200), (300, 37, 1024, 30), (40, 1, 4096, 1)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    jobs = []
    for j, (k, r, b, loss) in enumerate(shapes):
        rng = np.random.default_rng(100 + j)
        data = rng.integers(0, 256, (k, b), dtype=np.uint8)
        perm = rng.permutation(k)
        store = dev_tensor(data[perm])
        inv = np.argsort(perm)
        wc = leo.leo_encode_work_count(k, r)
        work = torch.zeros((wc, b), dtype=torch.uint8, device="cuda")
        dwc = leo.leo_decode_work_count(k, r)
        dwork = torch.zeros((dwc, b), dtype=torch.uint8, device="cuda")
        lo, lr = ol.benchmark_losses(k, r, loss, seed=9, trial=j)
        jobs.append(dict(k=k, r=r, b=b, data=data, store=store, inv=inv, work=work, dwork=dwork, lo=lo, lr=lr,
                         wc=wc, dwc=dwc))
    torch.cuda.synchronize()
    leo.set_async(True)
    try:
        for j, job in enumerate(jobs):  # every encode, alternating streams, nothing waited for
            leo.set_stream(streams[j % 2].cuda_stream)
            res = leo.leo_encode(job["b"], job["k"], job["r"], job["wc"],
                                 [job["store"][int(job["inv"][i])].data_ptr() for i in range(job["k"])],
                                 [job["work"][i].data_ptr() for i in reversed(range(job["wc"]))])
            assert res == leo.LeopardResult.Success, leo.last_error()
        for j, job in enumerate(jobs):  # decodes on the same streams as their encodes
            leo.set_stream(streams[j % 2].cuda_stream)
            wc = job["wc"]
            los, lrs = set(job["lo"]), set(job["lr"])
            res = leo.leo_decode(job["b"], job["k"], job["r"], job["dwc"],
                                 [None if i in los else job["store"][int(job["inv"][i])].data_ptr()
                                  for i in range(job["k"])],
                                 [None if i in lrs else job["work"][wc - 1 - i].data_ptr() for i in range(job["r"])],
                                 [job["dwork"][i].data_ptr() for i in range(job["dwc"])])
            assert res == leo.LeopardResult.Success, leo.last_error()
        torch.cuda.synchronize()
    finally:
        leo.set_async(False)
        leo.set_stream(None)
    for job in jobs:
        wc, r = job["wc"], job["r"]
        rec = job["work"].cpu().numpy()[wc - 1 - np.arange(r)]
        assert np.array_equal(rec, ol.oracle().encode(job["data"], r)), (job["k"], r)
        dw = job["dwork"].cpu().numpy()
        for i in job["lo"]:
            assert np.array_equal(dw[i], job["data"][i]), (job["k"], r, i)


# ------------------------------------------------------------- batches --

def _batch_objects(k, r, b, count, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, (k, b), dtype=np.uint8) for _ in range(count)]


@pytest.mark.parametrize("k,r,b,layout", [(128, 128, 4096, "slab"), (128, 128, 4096, "shuffled"),
                                          (100, 20, 64 * 37, "slab"), (100, 20, 64 * 37, "shuffled"),
                                          (200, 55, 1024, "slab"), (1000, 200, 256, "slab"), (16, 16, 256, "slab"),
                                          (100, 70, 512, "slab"), (1000, 200, 2560, "shuffled"),
                                          (300, 100, 640, "slab"), (1000, 1000, 320, "slab")])
def test_batch_encode_decode_match_oracle(leo, k, r, b, layout):
    """leo_amd_encode_batch / decode_batch (one launch over every object for
    GF(2^8); object by object otherwise) == independent calls == the oracle.
    Slab-laid objects travel in the kernel arguments (launches of <= 64
    objects: 16+16 runs 70 objects), shuffled piece orders through the
    uploaded argument blocks.  The decode batch mixes erasure patterns: full
    loss (half-position decoder), partial losses, and objects with lost
    recovery pieces.  GF(2^16) objects on narrow strips (m <= 256 encode,
    n <= 2048 decode) also run one grid per kernel; 20 of them span two
    decoder-state chunks (16 erasure patterns a launch pair)."""
    _batch_roundtrip(leo, k, r, b, layout, 70 if k == 16 else 20 if k + r > 256 else 5)


def _batch_roundtrip(leo, k, r, b, layout, count):
    """Encode batch == oracle on every object; decode batch with mixed erasure
    patterns (even objects full loss, odd ones partial) gives back every lost
    original."""
    objs = _batch_objects(k, r, b, count, k + r)
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    if layout == "slab":
        dev = [dev_tensor(d) for d in objs]
        rows = [list(range(k))] * count
    else:  # piece i of object o lives in row rows[o][i] of its tensor
        rows = [np.random.default_rng(o).permutation(k).tolist() for o in range(count)]
        dev = []
        for d, rw in zip(objs, rows):
            t = torch.empty((k, b), dtype=torch.uint8, device="cuda")
            t[torch.tensor(rw, device="cuda")] = dev_tensor(d)
            dev.append(t)
    works = [torch.zeros((wc, b), dtype=torch.uint8, device="cuda") for _ in range(count)]
    res = leo.leo_amd_encode_batch(b, k, r, wc, [[t[rw[i]].data_ptr() for i in range(k)] for t, rw in zip(dev, rows)],
                                   [[w[i].data_ptr() for i in range(wc)] for w in works])
    assert res == leo.LeopardResult.Success, leo.last_error()
    torch.cuda.synchronize()
    recs = [w[:r].cpu().numpy() for w in works]
    for d, rec in zip(objs, recs):
        assert np.array_equal(rec, ol.oracle().encode(d, r))
    rng = np.random.default_rng(7)
    pats = []
    for o in range(count):
        loss = min(k, r) if o % 2 == 0 else int(rng.integers(1, min(k, r) + 1))
        lo = sorted(rng.choice(k, loss, replace=False).tolist())
        lr = sorted(rng.choice(r, r - loss, replace=False).tolist())
        pats.append((set(lo), set(lr)))
    dworks = [torch.zeros((dwc, b), dtype=torch.uint8, device="cuda") for _ in range(count)]
    recd = [dev_tensor(x) for x in recs]
    res = leo.leo_amd_decode_batch(
        b, k, r, dwc,
        [[None if i in lo else dev[o][rows[o][i]].data_ptr() for i in range(k)] for o, (lo, _) in enumerate(pats)],
        [[None if i in lr else recd[o][i].data_ptr() for i in range(r)] for o, (_, lr) in enumerate(pats)],
        [[w[i].data_ptr() for i in range(dwc)] for w in dworks])
    assert res == leo.LeopardResult.Success, leo.last_error()
    torch.cuda.synchronize()
    for o, (lo, _) in enumerate(pats):
        got = dworks[o].cpu().numpy()
        for i in lo:
            assert np.array_equal(got[i], objs[o][i]), (o, i)


@pytest.mark.parametrize("b,count,layout", [(8192, 16, "slab"), (8192, 16, "shuffled"), (64 * 37, 56, "slab"),
                                            (61440, 3, "slab")])
def test_batch16_one_pass_grid_matches_oracle(leo, b, count, layout):
    """GF(2^16) batch decodes whose grid crosses the one-pass rule
    (leopard_amd.cpp batch16_one_pass: >= 4 workgroups of 16-unit strips per
    CU): k_dec16n_one_batch over every object in one grid, including a partial
    last strip (64 x 37-byte pieces: 18.5 strips), shuffled piece orders, and
    pieces >= 60 KiB in a batch of several objects."""
    assert (b // 8 + 15) // 16 * count >= 4 * 256
    _batch_roundtrip(leo, 1000, 200, b, layout, count)


_FORCED_BATCH16 = r"""
import sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, {tests!r})
import leopard_amd as leo, test_gpu_parity as t
assert leo.leo_init() == 0
for b, count in ((64 * 37, 4), (8192, 16)):
    t._batch_roundtrip(leo, 1000, 200, b, "slab", count)
print("forced ok")
"""


@pytest.mark.parametrize("one", ["0", "1"])
def test_batch16_forced_forms_match_oracle(one):
    """Both GF(2^16) batch-decode forms on both sides of the one-pass rule:
    the experiment build (lib/exp, LAMD_EXPERIMENT_ENV) with
    LEO_AMD_DEC16_BATCH_ONE=0 (two passes, also above the rule) or =1 (one
    pass, also on small grids with a partial last strip), in a child process."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    lib = os.path.join(repo, "leopard_amd", "lib", "exp", "libleopard_amd.so")
    assert os.path.exists(lib), "make -C leopard_amd builds lib/exp"
    env = dict(os.environ, LEOPARD_AMD_LIB=lib, LEO_AMD_DEC16_BATCH_ONE=one)
    p = subprocess.run([sys.executable, "-c", _FORCED_BATCH16.format(repo=repo, tests=here)], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0 and "forced ok" in p.stdout, (p.stdout[-2000:], p.stderr[-3000:])


@pytest.mark.parametrize("b", [64, 192, 256, 64 * 37, 65536 + 192])
def test_bitsliced_dense_tile_matches_oracle(leo, b):
    """The bit-sliced tile (rs_ff8_bs.hip) that runs slab batches of 128 + 128
    codes: encode against the oracle, full-loss decode back to the originals,
    on piece sizes that end in a partial 256-byte strip (64 / 128 / 192 bytes
    left) and in several launches' worth of objects (70 > 64 per launch)."""
    k = r = 128
    count = 3 if b > 4096 else 70
    objs = _batch_objects(k, r, b, count, b)
    dev = [dev_tensor(d) for d in objs]
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    works = [torch.zeros((wc, b), dtype=torch.uint8, device="cuda") for _ in range(count)]
    res = leo.leo_amd_encode_batch(b, k, r, wc, [[t[i].data_ptr() for i in range(k)] for t in dev],
                                   [[w[i].data_ptr() for i in range(wc)] for w in works])
    assert res == leo.LeopardResult.Success, leo.last_error()
    torch.cuda.synchronize()
    for o in range(count):  # every object of every launch
        assert np.array_equal(works[o][:r].cpu().numpy(), ol.oracle().encode(objs[o], r)), o
    dworks = [torch.zeros((dwc, b), dtype=torch.uint8, device="cuda") for _ in range(count)]
    res = leo.leo_amd_decode_batch(b, k, r, dwc, [[None] * k] * count,
                                   [[w[i].data_ptr() for i in range(r)] for w in works],
                                   [[w[i].data_ptr() for i in range(dwc)] for w in dworks])
    assert res == leo.LeopardResult.Success, leo.last_error()
    torch.cuda.synchronize()
    for o in range(count):
        assert torch.equal(dworks[o][:k], dev[o]), o


@pytest.mark.parametrize("b", [(512 << 10) + 192, 1 << 20])
def test_bitsliced_single_dense_calls(leo, b):
    """Single leo_encode / full-loss leo_decode calls of 128 + 128 codes on pieces
    of >= 512 KiB laid out as slabs run the bit-sliced tile as a one-object batch
    (leopard_amd.cpp dense_single_bs): encode against the oracle (a partial last
    strip at + 192 bytes), the full-loss decode back to the originals."""
    k = r = 128
    rng = np.random.default_rng(b)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    expect = ol.oracle().encode(data, r)
    got = gpu_encode(leo, data, r)
    assert np.array_equal(got, expect)
    dec = gpu_decode(leo, data, expect, list(range(k)), [])
    for i in range(k):
        assert np.array_equal(dec[i], data[i]), i


def test_bitsliced_headline_geometry(leo):
    """The benchmark's own launch: ONE encode-batch and ONE decode-batch launch
    over 64 objects of 128 + 128 x 65536 B laid out as slabs (bench.py
    `headline`, BASELINE configs[1]).  Four objects spread over the launch
    (first, two inside, last: different waves, rounds of the persistent grid
    and prefetch slots) are checked against the oracle; the full-loss decode
    of every object must give back its originals."""
    k = r = 128
    b, count = 65536, 64
    gen = torch.Generator(device="cuda").manual_seed(128)
    data = torch.randint(0, 256, (count, k, b), dtype=torch.uint8, device="cuda", generator=gen)
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    works = torch.zeros((count, wc, b), dtype=torch.uint8, device="cuda")
    res = leo.leo_amd_encode_batch(b, k, r, wc, [[data[o, i].data_ptr() for i in range(k)] for o in range(count)],
                                   [[works[o, i].data_ptr() for i in range(wc)] for o in range(count)])
    assert res == leo.LeopardResult.Success, leo.last_error()
    torch.cuda.synchronize()
    for o in (0, 21, 42, count - 1):
        assert np.array_equal(works[o, :r].cpu().numpy(), ol.oracle().encode(data[o].cpu().numpy(), r)), o
    dworks = torch.zeros((count, dwc, b), dtype=torch.uint8, device="cuda")
    res = leo.leo_amd_decode_batch(b, k, r, dwc, [[None] * k] * count,
                                   [[works[o, i].data_ptr() for i in range(r)] for o in range(count)],
                                   [[dworks[o, i].data_ptr() for i in range(dwc)] for o in range(count)])
    assert res == leo.LeopardResult.Success, leo.last_error()
    torch.cuda.synchronize()
    for o in range(count):
        assert torch.equal(dworks[o, :k], data[o]), o


def test_decoder_pattern_caches_evict_and_refill(leo):
    """The per-workspace erasure-pattern caches under eviction: 600 distinct
    GF(2^8) patterns (more than the 512 error-locator slots) and 20 GF(2^16)
    patterns (more than the 16 decoder-state slots) on one stream, then the
    earliest patterns again -- as single calls (for GF(2^8) the locator then
    travels by value) and as one batch.  Every decode must rebuild the lost
    originals; a stale slot would decode with another pattern's locator."""
    torch.cuda.synchronize()
    for k, r, b, npat, nbatch in [(100, 20, 64, 600, 16), (300, 100, 128, 20, 4)]:
        rng = np.random.default_rng(k + npat)
        data = rng.integers(0, 256, (k, b), dtype=np.uint8)
        rec = ol.oracle().encode(data, r)
        d_data, d_rec = dev_tensor(data), dev_tensor(rec)
        dwc = leo.leo_decode_work_count(k, r)
        pats, seen = [], set()
        while len(pats) < npat:
            loss = int(rng.integers(1, r + 1))
            lo = tuple(sorted(rng.choice(k, loss, replace=False).tolist()))
            lr = tuple(sorted(rng.choice(r, r - loss, replace=False).tolist()))
            if (lo, lr) not in seen:
                seen.add((lo, lr))
                pats.append((set(lo), set(lr)))
        order = list(range(npat)) + list(range(min(12, npat)))  # then the earliest (evicted) patterns again
        works = [torch.zeros((dwc, b), dtype=torch.uint8, device="cuda") for _ in order]

        def args(j, w):
            lo, lr = pats[j]
            return ([None if i in lo else d_data[i].data_ptr() for i in range(k)],
                    [None if i in lr else d_rec[i].data_ptr() for i in range(r)], [w[i].data_ptr() for i in range(dwc)])

        for j, w in zip(order, works):
            res = leo.leo_decode(b, k, r, dwc, *args(j, w))
            assert res == leo.LeopardResult.Success, leo.last_error()
        bworks = [torch.zeros((dwc, b), dtype=torch.uint8, device="cuda") for _ in range(nbatch)]
        ba = [args(j, w) for j, w in zip(range(nbatch), bworks)]
        res = leo.leo_amd_decode_batch(b, k, r, dwc, [a[0] for a in ba], [a[1] for a in ba], [a[2] for a in ba])
        assert res == leo.LeopardResult.Success, leo.last_error()
        torch.cuda.synchronize()
        for j, w in list(zip(order, works)) + list(zip(range(nbatch), bworks)):
            got = w.cpu().numpy()
            for i in pats[j][0]:
                assert np.array_equal(got[i], data[i]), (k, r, j, i)


def test_batch_full_loss_and_validation(leo):
    """The benchmark's batch (every original lost, the half-position decoder in
    one launch) and the batch validation rules."""
    k = r = 128
    b = 2048
    count = 4
    objs = _batch_objects(k, r, b, count, 3)
    dev = [dev_tensor(d) for d in objs]
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    works = [torch.zeros((wc, b), dtype=torch.uint8, device="cuda") for _ in range(count)]
    po = [[t[i].data_ptr() for i in range(k)] for t in dev]
    pw = [[w[i].data_ptr() for i in range(wc)] for w in works]
    assert leo.leo_amd_encode_batch(b, k, r, wc, po, pw) == leo.LeopardResult.Success
    dworks = [torch.zeros((dwc, b), dtype=torch.uint8, device="cuda") for _ in range(count)]
    pr = [[w[i].data_ptr() for i in range(r)] for w in works]
    pd = [[w[i].data_ptr() for i in range(dwc)] for w in dworks]
    assert leo.leo_amd_decode_batch(b, k, r, dwc, [[None] * k] * count, pr, pd) == leo.LeopardResult.Success
    torch.cuda.synchronize()
    for o in range(count):
        assert torch.equal(dworks[o][:k], dev[o])
    R = leo.LeopardResult
    # every object is validated before anything runs
    assert leo.leo_amd_encode_batch(b, k, r, wc - 1, po, pw) == R.InvalidCounts
    assert leo.leo_amd_encode_batch(b + 1, k, r, wc, po, pw) == R.InvalidSize
    short = [[None] * k] * count
    pr_bad = [list(x) for x in pr]
    pr_bad[2] = [None] * r  # object 2 received nothing
    assert leo.leo_amd_decode_batch(b, k, r, dwc, short, pr_bad, pd) == R.NeedMoreData
    assert leo.leo_amd_encode_batch(b, k, r, wc, [], []) == R.Success
    # a NULL recovery destination is rejected before anything runs (a single
    # leo_encode returns the same), never written through
    pw_bad = [list(x) for x in pw]
    pw_bad[1][5] = None
    assert leo.leo_amd_encode_batch(b, k, r, wc, po, pw_bad) == R.InvalidInput


@pytest.mark.parametrize("k,r,b,loss", [(128, 128, 1 << 16, 128), (100, 30, 64 * 1000, 17), (1000, 200, 1 << 13, 200),
                                        (9, 1, 1 << 14, 1), (128, 128, 1 << 16, 40), (300, 100, 1 << 15, 10),
                                        (1000, 200, 1 << 14, 200), (40, 10, 1 << 12, 5), (64, 1, 1 << 15, 1)])
def test_registered_host_memory_in_place(leo, k, r, b, loss):
    """leo_amd_register_host: host pieces in registered ranges are coded in place
    by the kernels (over PCIe, no staging); results equal the oracle and the
    decode rebuilds the originals, for one-slab and fragmented piece layouts,
    both fields and R = 1.  Unregistering falls back to staging."""
    data = ol.pcg_bytes(8, k, k, b)
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    work = np.zeros((wc, b), dtype=np.uint8)
    dwork = np.zeros((dwc, b), dtype=np.uint8)
    for arr in (data, work, dwork):
        assert leo.register_host(arr.ctypes.data, arr.nbytes) == leo.LeopardResult.Success, leo.last_error()
    try:
        res = leo.leo_encode(b, k, r, wc, [data[i].ctypes.data for i in range(k)],
                             [work[i].ctypes.data for i in range(wc)])
        assert res == leo.LeopardResult.Success, leo.last_error()
        assert np.array_equal(work[:r], ol.oracle().encode(data, r))
        rec = work[:r]
        lo, lr = ol.benchmark_losses(k, r, loss, seed=8, trial=b)
        res = leo.leo_decode(b, k, r, dwc, [None if i in lo else data[i].ctypes.data for i in range(k)],
                             [None if i in lr else rec[i].ctypes.data for i in range(r)],
                             [dwork[i].ctypes.data for i in range(dwc)])
        assert res == leo.LeopardResult.Success, leo.last_error()
        for i in lo:
            assert np.array_equal(dwork[i], data[i]), i
    finally:
        for arr in (data, work, dwork):
            assert leo.unregister_host(arr.ctypes.data) == leo.LeopardResult.Success
    assert leo.unregister_host(data.ctypes.data) == leo.LeopardResult.InvalidInput


# ------------------------------------------------------------ reentrancy --

def test_concurrent_host_threads_are_reentrant(leo):
    """The reference's encode/decode are reentrant (tables read-only after
    init, state on the stack: SURVEY.md 8(b), leopard.cpp:123-344).  Here each
    host thread has its own stream and scratch: 4 threads call leo_encode /
    leo_decode at once (ctypes drops the GIL) on host buffers and device
    buffers, GF(2^8) and GF(2^16) shapes, and every result must equal the
    oracle's."""
    import threading

    shapes = [(128, 128, 4096), (1000, 200, 256), (100, 20, 640), (300, 300, 128)]
    jobs = []
    for t, (k, r, b) in enumerate(shapes):
        rng = np.random.default_rng(100 + t)
        data = rng.integers(0, 256, (k, b), dtype=np.uint8)
        loss = min(k, r) // 2 + 1
        lo = sorted(rng.choice(k, loss, replace=False).tolist())
        lr = sorted(rng.choice(r, r - loss, replace=False).tolist())
        jobs.append(dict(k=k, r=r, b=b, data=data, rec=ol.oracle().encode(data, r), lo=lo, lr=lr))
    errors = []

    def worker(job, device):
        try:
            k, r, b = job["k"], job["r"], job["b"]
            wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
            for it in range(6):
                if device:
                    data = torch.from_numpy(job["data"]).cuda()
                    work = torch.zeros((wc, b), dtype=torch.uint8, device="cuda")
                    dwork = torch.zeros((dwc, b), dtype=torch.uint8, device="cuda")
                    ptr = lambda t, i: t[i].data_ptr()  # noqa: E731
                else:
                    data = job["data"]
                    work = np.zeros((wc, b), dtype=np.uint8)
                    dwork = np.zeros((dwc, b), dtype=np.uint8)
                    ptr = lambda t, i: t[i].ctypes.data  # noqa: E731
                torch.cuda.synchronize()
                res = leo.leo_encode(b, k, r, wc, [ptr(data, i) for i in range(k)], [ptr(work, i) for i in range(wc)])
                assert res == leo.LeopardResult.Success, leo.last_error()
                rec = work[:r].cpu().numpy() if device else work[:r]
                assert np.array_equal(rec, job["rec"]), ("encode", k, r, it, device)
                res = leo.leo_decode(b, k, r, dwc, [None if i in job["lo"] else ptr(data, i) for i in range(k)],
                                     [None if i in job["lr"] else ptr(work, i) for i in range(r)],
                                     [ptr(dwork, i) for i in range(dwc)])
                assert res == leo.LeopardResult.Success, leo.last_error()
                got = dwork.cpu().numpy() if device else dwork
                for i in job["lo"]:
                    assert np.array_equal(got[i], job["data"][i]), ("decode", k, r, it, device, i)
        except BaseException as e:  # noqa: BLE001 -- reported by the main thread
            errors.append(repr(e))

    for device in (False, True):
        threads = [threading.Thread(target=worker, args=(job, device)) for job in jobs]
        for th in threads:
            th.start()
        for th in threads:
            th.join(timeout=90)
        assert not any(th.is_alive() for th in threads), "a worker thread hung"
    assert not errors, errors


_FORCED_ENC16 = r"""
import sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, {tests!r})
import numpy as np
import leopard_amd as leo, test_gpu_parity as t, oracle_lib as ol
assert leo.leo_init() == 0
for k, r, b in {cases!r}:
    data = np.random.default_rng(k + r + b).integers(0, 256, (k, b), dtype=np.uint8)
    assert np.array_equal(t.gpu_encode(leo, data, r), ol.oracle().encode(data, r)), (k, r, b)
print("forced ok")
"""
ENC16_SPLIT_CASES = [(1000, 200, 2560), (300, 100, 64 * 37), (129, 127, 64), (700, 256, 128), (513, 200, 64 * 40)]


@pytest.mark.parametrize("k,r,b", ENC16_SPLIT_CASES)
def test_ff16_chunk_parallel_encode_matches_oracle(leo, k, r, b):
    """Single GF(2^16) encodes with m <= 256, several chunks and fewer 16-unit
    column strips than CUs (rs_ff16_small.hip k_enc16n_part + k_enc16n_comb):
    a zero-padded last chunk (K not a multiple of m), a partial last strip
    (64 x 37-byte pieces), m = 128 and m = 256."""
    rng = np.random.default_rng(k * 3 + r + b)
    data = rng.integers(0, 256, (k, b), dtype=np.uint8)
    assert np.array_equal(gpu_encode(leo, data, r), ol.oracle().encode(data, r))


@pytest.mark.parametrize("split", ["0", "1"])
def test_ff16_encode_forced_forms_match_oracle(split):
    """Both narrow GF(2^16) encode forms on both sides of the split rule: the
    experiment build with LEO_AMD_ENC16_SPLIT=0 (one kernel, also on few strips)
    or =1 (chunk-parallel, also on many strips), in a child process."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    lib = os.path.join(repo, "leopard_amd", "lib", "exp", "libleopard_amd.so")
    assert os.path.exists(lib), "make -C leopard_amd builds lib/exp"
    cases = ENC16_SPLIT_CASES + [(1000, 200, 65536), (300, 100, 8192)]
    env = dict(os.environ, LEOPARD_AMD_LIB=lib, LEO_AMD_ENC16_SPLIT=split)
    p = subprocess.run([sys.executable, "-c", _FORCED_ENC16.format(repo=repo, tests=here, cases=cases)], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0 and "forced ok" in p.stdout, (p.stdout[-2000:], p.stderr[-3000:])


_FORCED_MAT = r"""
import sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, {tests!r})
import leopard_amd as leo, test_gpu_parity as t
assert leo.leo_init() == 0
for c in {cases!r}:
    t.test_matrix_path_matches_oracle(leo, *c)
print("forced ok")
"""


@pytest.mark.parametrize("c,lb", [("1", "1"), ("1", "8"), ("2", "2"), ("2", "8"), ("4", "1"), ("4", "4")])
def test_matrix_kernel_forced_shapes_match_oracle(c, lb):
    """Every lane width C and output group LB of k_ff8_mat (experiment build,
    LEO_AMD_MAT_C / LEO_AMD_MAT_LB), on inputs per wave KI = 1 .. 16 and output
    counts that leave a partial group, in a child process."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    lib = os.path.join(repo, "leopard_amd", "lib", "exp", "libleopard_amd.so")
    assert os.path.exists(lib), "make -C leopard_amd builds lib/exp"
    cases = [(100, 10, 2560, 10, 0), (128, 128, 65536, 16, 0), (12, 3, 64 * 1000, 1, 0), (16, 16, 64, 1, 3),
             (32, 8, 65536, 4, 2), (200, 30, 256, 29, 0)]
    env = dict(os.environ, LEOPARD_AMD_LIB=lib, LEO_AMD_MAT_C=c, LEO_AMD_MAT_LB=lb)
    p = subprocess.run([sys.executable, "-c", _FORCED_MAT.format(repo=repo, tests=here, cases=cases)], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0 and "forced ok" in p.stdout, (p.stdout[-2000:], p.stderr[-3000:])
