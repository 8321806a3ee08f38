// SSZ hash_tree_root / computeSigningRoot pieces for the signing roots that feed the verifier
// (SURVEY.md 8(f) rank 3).  The SSZ library itself (@chainsafe/ssz 0.11.1, yarn.lock:661) is not
// vendored; what is restated is the consensus-spec merkleization its ContainerType.hashTreeRoot
// implements: every basic field is packed into one 32-byte chunk (uint64: little-endian, zero padded),
// a composite field contributes its own root, and the field chunks are merkleized as a binary tree
// zero-padded to the next power of two, each node = sha256(left || right).
#pragma once
#include "sha256.h"

namespace gbv {

// 32 bytes in memory order, read as 8 little-endian u32 words -> 8 big-endian SHA-256 words.
GBV_HD u32x8 ssz_chunk(const uint32_t* le) {
  u32x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = __builtin_bswap32(le[i]);
  return r;
}
// uint64 field (little-endian words lo, hi) -> its chunk.
GBV_HD u32x8 ssz_uint64_chunk(uint32_t lo, uint32_t hi) {
  u32x8 r = {0, 0, 0, 0, 0, 0, 0, 0};
  r[0] = __builtin_bswap32(lo);
  r[1] = __builtin_bswap32(hi);
  return r;
}
// zeroHash(1) = sha256(0^64), the root of an all-zero pair of chunks.
GBV_HD u32x8 ssz_zero_hash1() {
  u32x8 r = {0xf5a5fd42u, 0xd16a2030u, 0x2798ef6eu, 0xd309979bu, 0x43003d23u, 0x20d9f0e8u, 0xea9831a9u, 0x2759fb4bu};
  return r;
}

// hash_tree_root(phase0.AttestationData) (types/src/phase0/sszTypes.ts:247-256) from its 128-byte SSZ
// serialisation d (32 little-endian words): slot | index | beaconBlockRoot | source{epoch, root} |
// target{epoch, root}.  Five fields -> 8 leaves (3 zero); a Checkpoint is a two-leaf container.
// Eight digest64 nodes; (target, 0) and the constant zeroHash(1) stand in for the padding.
GBV_HD u32x8 ssz_attestation_data_root(const uint32_t d[32]) {
  u32x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  u32x8 src = sha256_node(ssz_uint64_chunk(d[12], d[13]), ssz_chunk(d + 14));
  u32x8 tgt = sha256_node(ssz_uint64_chunk(d[22], d[23]), ssz_chunk(d + 24));
  u32x8 n01 = sha256_node(ssz_uint64_chunk(d[0], d[1]), ssz_uint64_chunk(d[2], d[3]));
  u32x8 n23 = sha256_node(ssz_chunk(d + 4), src);
  u32x8 n45 = sha256_node(tgt, zero);
  return sha256_node(sha256_node(n01, n23), sha256_node(n45, ssz_zero_hash1()));
}

// computeSigningRoot (state-transition/src/util/signingRoot.ts:7-13):
// hash_tree_root(SigningData{objectRoot, domain}) = sha256(objectRoot || domain).
GBV_HD u32x8 ssz_signing_root(u32x8 object_root, u32x8 domain) { return sha256_node(object_root, domain); }

}  // namespace gbv
