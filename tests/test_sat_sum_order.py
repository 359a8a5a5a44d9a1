"""The certificate's S (pass.h): `tb_sum_total` adds the 64 shards one after another, saturating at
maxInt(u128), while `tb_sum_total_wave` adds them as an xor butterfly over a wave's lanes with a
sticky overflow flag. This checks on the host that both orders give min(true sum, maxInt) for
every lane, including sums that land exactly on maxInt, just past it, or overflow only at the root."""
import random

MAX = (1 << 128) - 1


def sequential(shards):
    s = 0
    for v in shards:
        r = s + v
        s = MAX if r > MAX else r
    return s


def butterfly(shards):
    vals, sat = list(shards), [False] * 64
    off = 1
    while off < 64:
        nv, ns = vals[:], sat[:]
        for lane in range(64):
            o = lane ^ off
            r = vals[lane] + vals[o]
            ns[lane] = sat[lane] or sat[o] or r > MAX
            nv[lane] = r & MAX
        vals, sat = nv, ns
        off <<= 1
    return [MAX if s else v for v, s in zip(vals, sat)]


def cases():
    rng = random.Random(5)
    yield [0] * 64
    yield [rng.getrandbits(60) for _ in range(64)]
    exact = [rng.getrandbits(120) for _ in range(63)]
    yield exact + [MAX - sum(exact)]                      # lands exactly on maxInt
    yield exact + [MAX - sum(exact) + 1]                  # one past it
    yield [MAX // 2 + 1] + [0] * 62 + [MAX // 2 + 1]      # overflows only at the root
    yield [MAX] + [rng.getrandbits(64) for _ in range(63)]
    for _ in range(200):
        bits = rng.choice([32, 64, 100, 122, 126, 127, 128])
        yield [rng.getrandbits(bits) for _ in range(64)]


def test_butterfly_equals_sequential_saturating_sum():
    for shards in cases():
        want = sequential(shards)
        assert min(sum(shards), MAX) == want
        assert butterfly(shards) == [want] * 64
