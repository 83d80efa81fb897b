// bcw_parse.h -- the record payload parsers shared by the decode (bcw_decode.hip) and the point reads
// (bcw_read.hip): Go encoding/binary.Uvarint with DecodeUvarint's error mapping (utils.go:51-57),
// RecordFromBytes (record.go:140-239) and HintRecord.Decode (hint.go:50-84), over any byte accessor
// `rd(pos)` of the payload.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bcw.h"

namespace bcw {

// Go encoding/binary.Uvarint over a byte accessor; DecodeUvarint maps errors to (0,0).
template <typename RD>
__device__ __forceinline__ uint64_t uvarint(RD& rd, uint64_t pos, uint64_t len, uint32_t& used) {
  uint64_t x = 0;
  uint32_t s = 0;
  // rolled: each call site inlines the reader (its fragment-walk fallback included), so an unrolled loop
  // multiplies the code (k_records: 17.7 k lines of ISA unrolled, 4.7 k rolled; SGPR spills 4-6x fewer)
#pragma unroll 1
  for (uint32_t i = 0; pos + i < len; ++i) {
    if (i == 10) { used = 0; return 0; }
    const uint32_t b = rd(pos + i);
    if (b < 0x80u) {
      if (i == 9 && b > 1u) { used = 0; return 0; }
      used = i + 1;
      return x | ((uint64_t)b << s);
    }
    x |= (uint64_t)(b & 0x7fu) << s;
    s += 7;
  }
  used = 0;
  return 0;
}

template <typename RD>
__device__ __forceinline__ void parse_record(const bcw_decode_params& p, RD& rd, uint64_t len, uint8_t& status,
                                             uint8_t& hdr, uint8_t& flags, uint8_t& etag_off, uint64_t& key_len,
                                             uint64_t& val_len, uint64_t& meta_len, uint64_t& expire, uint64_t& aux0,
                                             uint64_t& aux1) {
  uint32_t used;
  status = BCW_ST_OK;
  hdr = flags = etag_off = 0;
  key_len = val_len = meta_len = expire = aux0 = aux1 = 0;
  if (p.mode == BCW_MODE_RECORD) {
    // RecordFromBytes, record.go:140-239
    const uint64_t min_hdr = 1ull + p.ns_size + 1ull + 3ull;
    if (len < min_hdr) { status = BCW_ST_INVALID; return; }
    const uint64_t header = rd(0);
    uint64_t o = 1 + p.ns_size;
    const uint32_t flag = rd(o);
    ++o;
    key_len = uvarint(rd, o, len, used); o += used;
    val_len = uvarint(rd, o, len, used); o += used;
    meta_len = uvarint(rd, o, len, used); o += used;
    const uint64_t etag_len = (flag & 1u) ? 0 : p.etag_size;
    uint64_t expire_size = 0;
    hdr = (uint8_t)header; flags = (uint8_t)flag; etag_off = (uint8_t)o;
    if ((flag & 2u) == 0) {
      if (o + etag_len > len) { status = BCW_ST_PANIC; return; }  // data[offset+etagLen:] (record.go:186)
      expire = uvarint(rd, o + etag_len, len, used);
      expire_size = used;
      expire += p.base_time;
    }
    const int64_t cur_hdr = (int64_t)o + (int64_t)etag_len + (int64_t)expire_size;
    const int64_t cur_total = cur_hdr + (int64_t)(key_len + val_len + meta_len);
    if ((uint64_t)cur_hdr != header || cur_total != (int64_t)len) { status = BCW_ST_INVALID; return; }
    const uint64_t s1 = key_len + val_len;
    const uint64_t s2 = s1 + meta_len;
    const bool wrapped = (s1 < key_len) || (s2 < s1);
    if ((int64_t)key_len < 0 || (int64_t)val_len < 0 || (int64_t)meta_len < 0 || wrapped) status = BCW_ST_PANIC;
    else if (key_len > 0xffffffffull || val_len > 0xffffffffull || meta_len > 0xffffffffull || len > 0xffffffffull)
      status = BCW_ST_UNSUPPORTED;
  } else {
    // HintRecord.Decode, hint.go:50-84
    if (len < (uint64_t)p.ns_size + 5ull) { status = BCW_ST_INVALID; return; }
    int64_t o = p.ns_size;
    key_len = uvarint(rd, (uint64_t)o, len, used);
    o += used;
    const int64_t key_off = o;
    o = (int64_t)((uint64_t)o + key_len);
    hdr = (uint8_t)key_off;
    if (o < 0 || o > (int64_t)len) { status = BCW_ST_PANIC; return; }
    expire = uvarint(rd, (uint64_t)o, len, used); o += used;  // fid
    aux0 = uvarint(rd, (uint64_t)o, len, used); o += used;    // off
    aux1 = uvarint(rd, (uint64_t)o, len, used); o += used;    // size
    if (o != (int64_t)len) status = BCW_ST_INVALID;
    else if ((int64_t)key_len < 0) status = BCW_ST_PANIC;
  }
}

}  // namespace bcw
