// libcessec on-chain records: the SCALE bytes the codec's outputs become on chain. Host only.
//
//   FileBank::upload_declaration(origin, file_hash: Hash,
//                                deal_info: BoundedVec<SegmentList<T>, T::SegmentCount>,
//                                user_brief: UserBrief<T>)      c-pallets/file-bank/src/lib.rs:423-428
//   SegmentList { hash: Hash, fragment_list: BoundedVec<Hash, FragmentCount> }   types.rs:13-16
//   UserBrief { user: AccountId, file_name: BoundedVec<u8, NameStrLimit>,
//               bucket_name: BoundedVec<u8, NameStrLimit> }                      types.rs:105-109
//   Hash([u8; 64])                                   primitives/common/src/lib.rs:16
//   SEGMENT_COUNT = 1000, FRAGMENT_COUNT = 3         runtime/src/lib.rs:1026-1027
//   NameStrLimit = 63, NameMinLength = 3             runtime/src/lib.rs:1041,1051
//   FileBank = pallet index 60, upload_declaration = call index 0
//                                                    runtime/src/lib.rs:1532, lib.rs:419
//   from_shard_id: first 64 of 68 bytes               primitives/common/src/lib.rs:45-49
//   upload_filler(tee_worker: AccountId, filler_list: Vec<FillerInfo>)   call_index(8)
//                                                    lib.rs:795-833
//   FillerInfo { block_num: u32, miner_address: AccountId, filler_hash: Hash }  types.rs:82-86
//   UploadFillerLimit = 10                           runtime/src/lib.rs:1033
//   generate_restoral_order(file_hash, restoral_fragment)            call_index(13) lib.rs:940-984
//   claim_restoral_order(restoral_fragment)                          call_index(14) lib.rs:986-1014
//   claim_restoral_exist_order(miner, file_hash, restoral_fragment)  call_index(15) lib.rs:1016-1070
//   restoral_order_complete(fragment_hash)                           call_index(16) lib.rs:1072-1122
//   Audit::random_number(seed): MyRandomness::random(&(MyPalletId, seed).encode()), then the
//     output's first 8 bytes decoded as u64          c-pallets/audit/src/lib.rs:1067-1076
//   audit MyPalletId = SegbkPalletId = PalletId(*b"rewardpt")   runtime/src/lib.rs:984,1004
//
// SCALE (parity-scale-codec): a fixed array [u8; N] is its N bytes; a Vec / BoundedVec is a
// compact length then its items; a struct is its fields in order; AccountId32 is 32 bytes.
// Compact u32: < 2^6 one byte (n << 2), < 2^14 two bytes LE ((n << 2) | 1), < 2^30 four bytes
// LE ((n << 2) | 2), else 0x03 + the 4 bytes.
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cess_ec.h"

namespace cec {
int set_error(int code, const std::string& msg);
}

namespace {

void put_compact(std::vector<uint8_t>& o, uint32_t n) {
  if (n < (1u << 6)) {
    o.push_back((uint8_t)(n << 2));
  } else if (n < (1u << 14)) {
    const uint32_t v = (n << 2) | 1u;
    o.push_back((uint8_t)v);
    o.push_back((uint8_t)(v >> 8));
  } else if (n < (1u << 30)) {
    const uint32_t v = (n << 2) | 2u;
    for (int i = 0; i < 4; ++i) o.push_back((uint8_t)(v >> (8 * i)));
  } else {
    o.push_back(3);
    for (int i = 0; i < 4; ++i) o.push_back((uint8_t)(n >> (8 * i)));
  }
}

int check_hex(const uint8_t* h, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const uint8_t c = h[i];
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f')))
      return cec::set_error(CEC_EINVAL, "hash is not 64 lowercase hex characters");
  }
  return CEC_OK;
}

int deal_info(std::vector<uint8_t>& o, const uint8_t* seg_hex, const uint8_t* frag_hex,
              size_t nseg, size_t nfrag) {
  if (nseg && (!seg_hex || !frag_hex)) return cec::set_error(CEC_EINVAL, "null hashes");
  if (nseg > CEC_SEGMENT_COUNT)
    return cec::set_error(CEC_ESEGCOUNT, "deal_info holds at most SegmentCount = 1000 segments "
                                         "(16,000 MiB): split the file");
  // check_file_spec (c-pallets/file-bank/src/functions.rs:4-11): every fragment_list holds
  // exactly FragmentCount hashes, or upload_declaration fails with SpecError
  if (nfrag != CEC_FRAGMENT_COUNT)
    return cec::set_error(CEC_EINVAL, "fragment_list holds exactly FragmentCount = 3 hashes "
                                      "(check_file_spec)");
  int rc = check_hex(seg_hex, nseg * 64);
  if (!rc) rc = check_hex(frag_hex, nseg * nfrag * 64);
  if (rc) return rc;
  put_compact(o, (uint32_t)nseg);
  for (size_t s = 0; s < nseg; ++s) {
    o.insert(o.end(), seg_hex + s * 64, seg_hex + (s + 1) * 64);
    put_compact(o, (uint32_t)nfrag);
    const uint8_t* f = frag_hex + s * nfrag * 64;
    o.insert(o.end(), f, f + nfrag * 64);
  }
  return CEC_OK;
}

void put_u32(std::vector<uint8_t>& o, uint32_t v) {
  for (int i = 0; i < 4; ++i) o.push_back((uint8_t)(v >> (8 * i)));
}

// a Hash argument: 64 lowercase hex bytes, no length prefix
int put_hash(std::vector<uint8_t>& o, const uint8_t* hex) {
  if (!hex) return cec::set_error(CEC_EINVAL, "null hash");
  int rc = check_hex(hex, 64);
  if (rc) return rc;
  o.insert(o.end(), hex, hex + 64);
  return CEC_OK;
}

int put_account(std::vector<uint8_t>& o, const uint8_t* acct) {
  if (!acct) return cec::set_error(CEC_EINVAL, "null account");
  o.insert(o.end(), acct, acct + 32);  // AccountId32: 32 bytes, no prefix
  return CEC_OK;
}

int emit(const std::vector<uint8_t>& o, uint8_t* out, size_t out_cap, size_t* out_len) {
  if (out_len) *out_len = o.size();
  if (!out) return CEC_OK;  // size query
  if (out_cap < o.size()) return cec::set_error(CEC_EINVAL, "output buffer too small");
  std::memcpy(out, o.data(), o.size());
  return CEC_OK;
}

}  // namespace

extern "C" {

int cec_scale_compact(uint32_t n, uint8_t* out, size_t out_cap, size_t* out_len) {
  std::vector<uint8_t> o;
  put_compact(o, n);
  return emit(o, out, out_cap, out_len);
}

int cec_scale_deal_info(const uint8_t* seg_hex, const uint8_t* frag_hex, size_t nseg,
                        size_t nfrag, uint8_t* out, size_t out_cap, size_t* out_len) {
  std::vector<uint8_t> o;
  int rc = deal_info(o, seg_hex, frag_hex, nseg, nfrag);
  if (rc) return rc;
  return emit(o, out, out_cap, out_len);
}

int cec_scale_upload_declaration(const uint8_t* file_hash_hex, const uint8_t* seg_hex,
                                 const uint8_t* frag_hex, size_t nseg, size_t nfrag,
                                 const uint8_t* account, const uint8_t* file_name,
                                 size_t file_name_len, const uint8_t* bucket_name,
                                 size_t bucket_name_len, uint8_t* out, size_t out_cap,
                                 size_t* out_len) {
  if (!file_hash_hex || !account || (file_name_len && !file_name) ||
      (bucket_name_len && !bucket_name))
    return cec::set_error(CEC_EINVAL, "null argument");
  if (file_name_len < CEC_NAME_MIN || file_name_len > CEC_NAME_MAX ||
      bucket_name_len < CEC_NAME_MIN || bucket_name_len > CEC_NAME_MAX)
    return cec::set_error(CEC_EINVAL, "file and bucket names take 3..63 bytes "
                                      "(NameMinLength, NameStrLimit)");
  int rc = check_hex(file_hash_hex, 64);
  if (rc) return rc;
  std::vector<uint8_t> o;
  o.push_back(CEC_FILEBANK_PALLET);
  o.push_back(CEC_CALL_UPLOAD_DECLARATION);
  o.insert(o.end(), file_hash_hex, file_hash_hex + 64);
  rc = deal_info(o, seg_hex, frag_hex, nseg, nfrag);
  if (rc) return rc;
  o.insert(o.end(), account, account + 32);
  put_compact(o, (uint32_t)file_name_len);
  o.insert(o.end(), file_name, file_name + file_name_len);
  put_compact(o, (uint32_t)bucket_name_len);
  o.insert(o.end(), bucket_name, bucket_name + bucket_name_len);
  return emit(o, out, out_cap, out_len);
}

int cec_scale_upload_filler(const uint8_t* tee_worker, const uint32_t* block_num,
                            const uint8_t* miners, const uint8_t* filler_hex, size_t n,
                            uint8_t* out, size_t out_cap, size_t* out_len) {
  if (n > CEC_UPLOAD_FILLER_LIMIT)
    return cec::set_error(CEC_EINVAL, "filler_list holds at most UploadFillerLimit = 10 fillers "
                                      "(LengthExceedsLimit)");
  if (n && (!block_num || !miners || !filler_hex))
    return cec::set_error(CEC_EINVAL, "null filler arrays");
  std::vector<uint8_t> o;
  o.push_back(CEC_FILEBANK_PALLET);
  o.push_back(CEC_CALL_UPLOAD_FILLER);
  int rc = put_account(o, tee_worker);
  if (rc) return rc;
  put_compact(o, (uint32_t)n);
  for (size_t i = 0; i < n; ++i) {  // FillerInfo: block_num, miner_address, filler_hash
    put_u32(o, block_num[i]);
    put_account(o, miners + 32 * i);
    if ((rc = put_hash(o, filler_hex + 64 * i))) return rc;
  }
  return emit(o, out, out_cap, out_len);
}

int cec_scale_generate_restoral_order(const uint8_t* file_hash_hex, const uint8_t* fragment_hex,
                                      uint8_t* out, size_t out_cap, size_t* out_len) {
  std::vector<uint8_t> o{CEC_FILEBANK_PALLET, CEC_CALL_GENERATE_RESTORAL_ORDER};
  int rc = put_hash(o, file_hash_hex);
  if (!rc) rc = put_hash(o, fragment_hex);
  return rc ? rc : emit(o, out, out_cap, out_len);
}

int cec_scale_claim_restoral_order(const uint8_t* fragment_hex, uint8_t* out, size_t out_cap,
                                   size_t* out_len) {
  std::vector<uint8_t> o{CEC_FILEBANK_PALLET, CEC_CALL_CLAIM_RESTORAL_ORDER};
  int rc = put_hash(o, fragment_hex);
  return rc ? rc : emit(o, out, out_cap, out_len);
}

int cec_scale_claim_restoral_exist_order(const uint8_t* miner, const uint8_t* file_hash_hex,
                                         const uint8_t* fragment_hex, uint8_t* out,
                                         size_t out_cap, size_t* out_len) {
  std::vector<uint8_t> o{CEC_FILEBANK_PALLET, CEC_CALL_CLAIM_RESTORAL_EXIST_ORDER};
  int rc = put_account(o, miner);
  if (!rc) rc = put_hash(o, file_hash_hex);
  if (!rc) rc = put_hash(o, fragment_hex);
  return rc ? rc : emit(o, out, out_cap, out_len);
}

int cec_scale_restoral_order_complete(const uint8_t* fragment_hex, uint8_t* out, size_t out_cap,
                                      size_t* out_len) {
  std::vector<uint8_t> o{CEC_FILEBANK_PALLET, CEC_CALL_RESTORAL_ORDER_COMPLETE};
  int rc = put_hash(o, fragment_hex);
  return rc ? rc : emit(o, out, out_cap, out_len);
}

int cec_audit_random_subject(const uint8_t* pallet_id, uint32_t seed, uint8_t* out12) {
  if (!pallet_id || !out12) return cec::set_error(CEC_EINVAL, "null");
  // SCALE of the tuple (PalletId, u32): PalletId([u8; 8]) is its 8 bytes, then u32 LE
  std::memcpy(out12, pallet_id, 8);
  for (int i = 0; i < 4; ++i) out12[8 + i] = (uint8_t)(seed >> (8 * i));
  return CEC_OK;
}

// NetSnapShot.random_list (c-pallets/audit/src/lib.rs:966-974): for seed = now + 1, now + 2, ...
// generate_challenge_random(seed) (:1079-1096) asks the randomness for the subject
// (MyPalletId, seed + 1) and returns the first 20 bytes of the H256 the output decodes as (an H256
// is 32 bytes, so its loop ends on the first try); values already in the list are skipped.
int cec_challenge_random_list(const uint8_t* randomness, size_t nrand, uint32_t need,
                              uint8_t* out, size_t* used) {
  if ((nrand && !randomness) || (need && !out)) return cec::set_error(CEC_EINVAL, "null");
  constexpr size_t kB = CEC_CHALLENGE_RANDOM_BYTES;
  uint32_t got = 0;
  size_t i = 0;
  for (; i < nrand && got < need; ++i) {
    const uint8_t* v = randomness + i * CEC_RANDOMNESS_BYTES;
    bool seen = false;
    for (uint32_t q = 0; q < got && !seen; ++q) seen = std::memcmp(out + q * kB, v, kB) == 0;
    if (!seen) std::memcpy(out + (got++) * kB, v, kB);
  }
  if (used) *used = i;
  if (got < need)
    return cec::set_error(CEC_EINVAL, "randomness stream exhausted before `need` values");
  return CEC_OK;
}

int cec_audit_random_u64(const uint8_t* randomness, size_t len, uint64_t* out) {
  if (!randomness || !out) return cec::set_error(CEC_EINVAL, "null");
  if (len < 8) return cec::set_error(CEC_EINVAL, "u64 decode needs at least 8 bytes");
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = v << 8 | randomness[i];
  *out = v;
  return CEC_OK;
}

int cec_shard_id(const uint8_t* hash_hex, uint32_t index, uint8_t* out68) {
  if (!hash_hex || !out68) return cec::set_error(CEC_EINVAL, "null");
  if (index > 999) return cec::set_error(CEC_EINVAL, "shard index takes three digits");
  int rc = check_hex(hash_hex, 64);
  if (rc) return rc;
  std::memcpy(out68, hash_hex, 64);
  out68[64] = '-';
  out68[65] = (uint8_t)('0' + index / 100);
  out68[66] = (uint8_t)('0' + index / 10 % 10);
  out68[67] = (uint8_t)('0' + index % 10);
  return CEC_OK;
}

int cec_hash_from_shard_id(const uint8_t* shard_id68, uint8_t* hash_hex_out) {
  if (!shard_id68 || !hash_hex_out) return cec::set_error(CEC_EINVAL, "null");
  std::memcpy(hash_hex_out, shard_id68, 64);
  return CEC_OK;
}

}  // extern "C"
