"""vsr.checksum (src/vsr/checksum.zig) as computed by the engine library's host-side
tbgpu_checksum (Aegis-128L MAC, zero key), pinned by the reference's own vectors: the two test
vectors (:83-101) and the "checksum stability" change detector (:135-184), whose 896 cases include
Zig's Xoshiro256 stream for seed 92 (restated below: SplitMix64 seeding, xoshiro256++ output, fill
in little-endian 8-byte words).  CPU only: the function touches no device."""
from tigerbeetle_amd._lib import checksum

M64 = (1 << 64) - 1


def byteswap128(x):
    return int.from_bytes(x.to_bytes(16, "big"), "little")


def test_reference_vectors():
    assert checksum(b"\0" * 16) == byteswap128(0xf72ad48dd05dd1656133101cd4be3a26)
    assert checksum(b"") == byteswap128(0x83cc600dc4e3e7e62d4055826174f149)


class Xoshiro256:
    """Zig 0.11 std.rand.Xoshiro256 (xoshiro256++), seeded through SplitMix64."""

    def __init__(self, seed):
        s = seed
        self.s = []
        for _ in range(4):
            s = (s + 0x9E3779B97F4A7C15) & M64
            z = s
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
            self.s.append(z ^ (z >> 31))

    def next(self):
        s = self.s
        rotl = lambda x, k: ((x << k) | (x >> (64 - k))) & M64
        r = (rotl((s[0] + s[3]) & M64, 23) + s[0]) & M64
        t = (s[1] << 17) & M64
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = rotl(s[3], 45)
        return r

    def fill(self, n):
        out = bytearray()
        while len(out) + 8 <= n:
            out += self.next().to_bytes(8, "little")
        if len(out) < n:
            out += self.next().to_bytes(8, "little")[:n - len(out)]
        return bytes(out)


def test_checksum_stability():
    cases = []
    for sub in range(128):  # zeros of various lengths
        cases.append(checksum(b"\0" * sub))
    for sub in range(64 * 8):  # 64 bytes with exactly one bit set
        m = bytearray(64)
        m[sub // 8] = 1 << (sub % 8)
        cases.append(checksum(bytes(m)))
    prng = Xoshiro256(92)
    for sub in range(256):  # pseudo-random data of various lengths
        cases.append(checksum(prng.fill(sub + 13)))
    assert len(set(cases)) == 896 and 0 not in cases
    blob = b"".join(c.to_bytes(16, "little") for c in cases)
    assert checksum(blob) == 0x82dcaacf4875b279446825b6830d1263
