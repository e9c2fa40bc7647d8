/*
 * tdb_oracle.c -- TEST INFRASTRUCTURE ONLY (see tdb_oracle.h).
 *
 * Plain-C restatement of TileDB's tile filter pipeline for the six filters
 * the MI355X engine implements (byteshuffle, bitshuffle, bit-width reduction,
 * positive delta, double delta, fixed-size RLE) plus the pass-through cases
 * (NOOP, NO_COMPRESSION, BWR/PD on non-integer types, datetime < v20).
 * Each routine cites the reference file:line it follows (paths relative to
 * the TileDB source root).  Forward (filter) routines exist only to produce
 * test fixtures; reverse (unfilter) routines are the parity checker.
 *
 * Byte/bit shuffles restate c-blosc2 v2.21.3 (ports/blosc2/vcpkg.json:3),
 * which TileDB calls at byteshuffle_filter.cc:97,154 and
 * bitshuffle_filter.cc:146-149 but does not vendor.
 */
#include "tdb_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* datatypes (tiledb/sm/enums/datatype.h:67-140, 342-415)                   */
/* ------------------------------------------------------------------------ */
uint64_t oracle_datatype_size(uint8_t dt) {
  switch (dt) {
    case TDBG_INT32: case TDBG_FLOAT32: case TDBG_UINT32:
    case TDBG_STRING_UTF32: case TDBG_STRING_UCS4:
      return 4;
    case TDBG_INT64: case TDBG_FLOAT64: case TDBG_UINT64:
      return 8;
    case TDBG_INT16: case TDBG_UINT16: case TDBG_STRING_UTF16:
    case TDBG_STRING_UCS2:
      return 2;
    default:
      if (dt >= 18 && dt <= 39) return 8; /* DATETIME_* / TIME_* */
      return 1; /* CHAR, INT8, UINT8, strings, ANY, BLOB, BOOL, GEOM */
  }
}

static int is_datetime_or_time(uint8_t dt) { return dt >= 18 && dt <= 39; }

/* Integer view of a filter datatype: width in bytes, signedness, and whether
 * the filter is active.  BWR: bit_width_reduction_filter.cc:288-350.
 * PD: positive_delta_filter.cc:262-322. */
typedef struct { int active; uint32_t w; int sgn; } ival_t;

static ival_t bwr_type(uint8_t dt, uint32_t version) {
  ival_t r = {0, 0, 0};
  switch (dt) {
    case TDBG_INT16: r.active = 1; r.w = 2; r.sgn = 1; break;
    case TDBG_UINT16: r.active = 1; r.w = 2; r.sgn = 0; break;
    case TDBG_INT32: r.active = 1; r.w = 4; r.sgn = 1; break;
    case TDBG_UINT32: r.active = 1; r.w = 4; r.sgn = 0; break;
    case TDBG_INT64: r.active = 1; r.w = 8; r.sgn = 1; break;
    case TDBG_UINT64: r.active = 1; r.w = 8; r.sgn = 0; break;
    default:
      if (is_datetime_or_time(dt) && version >= 20) {
        r.active = 1; r.w = 8; r.sgn = 1;
      }
  }
  return r;
}

static ival_t pd_type(uint8_t dt, uint32_t version) {
  ival_t r = {0, 0, 0};
  switch (dt) {
    case TDBG_INT8: r.active = 1; r.w = 1; r.sgn = 1; break;
    case TDBG_BLOB: case TDBG_GEOM_WKB: case TDBG_GEOM_WKT: case TDBG_BOOL:
    case TDBG_UINT8: r.active = 1; r.w = 1; r.sgn = 0; break;
    case TDBG_INT16: r.active = 1; r.w = 2; r.sgn = 1; break;
    case TDBG_UINT16: r.active = 1; r.w = 2; r.sgn = 0; break;
    case TDBG_INT32: r.active = 1; r.w = 4; r.sgn = 1; break;
    case TDBG_UINT32: r.active = 1; r.w = 4; r.sgn = 0; break;
    case TDBG_INT64: r.active = 1; r.w = 8; r.sgn = 1; break;
    case TDBG_UINT64: r.active = 1; r.w = 8; r.sgn = 0; break;
    default:
      if (is_datetime_or_time(dt) && version >= 20) {
        r.active = 1; r.w = 8; r.sgn = 1;
      }
  }
  return r;
}

/* DoubleDelta::decompress/compress type switch, dd_compressor.cc:63-200. */
static int dd_type(uint8_t dt, ival_t* r) {
  r->active = 1;
  switch (dt) {
    case TDBG_INT8: case TDBG_CHAR: r->w = 1; r->sgn = 1; return TDBG_OK;
    case TDBG_BLOB: case TDBG_GEOM_WKB: case TDBG_GEOM_WKT: case TDBG_BOOL:
    case TDBG_UINT8: r->w = 1; r->sgn = 0; return TDBG_OK;
    case TDBG_INT16: r->w = 2; r->sgn = 1; return TDBG_OK;
    case TDBG_UINT16: r->w = 2; r->sgn = 0; return TDBG_OK;
    case TDBG_INT32: r->w = 4; r->sgn = 1; return TDBG_OK;
    case TDBG_UINT32: r->w = 4; r->sgn = 0; return TDBG_OK;
    case TDBG_INT64: r->w = 8; r->sgn = 1; return TDBG_OK;
    case TDBG_UINT64: r->w = 8; r->sgn = 0; return TDBG_OK;
    case TDBG_FLOAT32: case TDBG_FLOAT64: return TDBG_E_DD_TYPE;
    default:
      if (is_datetime_or_time(dt)) { r->w = 8; r->sgn = 1; return TDBG_OK; }
      if ((dt >= TDBG_STRING_ASCII && dt <= TDBG_STRING_UCS4) || dt == TDBG_ANY) {
        r->w = 1; r->sgn = 0; return TDBG_OK;
      }
      return TDBG_E_DD_TYPE;
  }
}

static uint64_t ld(const uint8_t* p, uint32_t w) {
  uint64_t v = 0;
  memcpy(&v, p, w); /* little-endian host */
  return v;
}
static void st(uint8_t* p, uint64_t v, uint32_t w) { memcpy(p, &v, w); }
static uint64_t mask_w(uint32_t w) { return w >= 8 ? ~0ull : ((1ull << (8 * w)) - 1); }
static int64_t sext(uint64_t v, uint32_t w) {
  if (w >= 8) return (int64_t)v;
  uint32_t sh = 64 - 8 * w;
  return (int64_t)(v << sh) >> sh;
}

/* ------------------------------------------------------------------------ */
/* pipeline descriptor                                                       */
/* ------------------------------------------------------------------------ */
static uint8_t output_datatype(const oracle_filter* f, uint8_t in) {
  /* CompressionFilter::output_datatype compression_filter.cc:729-738 */
  if ((f->type == TDBG_FILTER_DOUBLE_DELTA || f->type == TDBG_FILTER_DELTA) &&
      f->reinterpret != TDBG_ANY)
    return f->reinterpret;
  /* XORFilter::output_datatype xor_filter.cc:63-78: the signed integer of
   * the input's width (other widths throw; kept as is, the filter fails) */
  /* FloatScalingFilter::output_datatype float_scaling_filter.cc:313-327 */
  if (f->type == TDBG_FILTER_SCALE_FLOAT) {
    switch (f->byte_width) {
      case 1: return TDBG_INT8;
      case 2: return TDBG_INT16;
      case 4: return TDBG_INT32;
      case 8: return TDBG_INT64;
      default: return in;
    }
  }
  if (f->type == TDBG_FILTER_XOR) {
    switch (oracle_datatype_size(in)) {
      case 1: return TDBG_INT8;
      case 2: return TDBG_INT16;
      case 4: return TDBG_INT32;
      case 8: return TDBG_INT64;
      default: return in;
    }
  }
  return in;
}

/* XORFilter::xor_part / unxor_part (xor_filter.cc:149-177, 260-286):
 * out[0] = in[0]; forward out[j] = in[j] ^ in[j-1], reverse
 * out[j] = in[j] ^ out[j-1], over the part's n/ts whole elements.  The
 * reference writes nothing for a part's n % ts tail bytes (its forward output
 * holds whatever the fresh buffer held); here the forward zero-fills them and
 * the reverse leaves them untouched, so tails are parity-unpinned. */
static void xor_part(int inverse, uint32_t ts, const uint8_t* in, uint64_t n, uint8_t* out) {
  uint64_t ne = n / ts, prev = 0;
  for (uint64_t j = 0; j < ne; j++) {
    uint64_t v = ld(in + j * ts, ts), o = j == 0 ? v : v ^ prev;
    st(out + j * ts, o, ts);
    prev = inverse ? o : v;
  }
}

/* FloatScalingFilter forward (float_scaling_filter.cc:60-99): W(round((x -
 * (T)offset) / (T)scale)) in T arithmetic; reverse (:164-197):
 * (T)(scale * (double)(T)w + offset), double multiply and add, not fused. */
static void fscale_fwd(uint32_t ts, uint32_t bw, double sc, double of, const uint8_t* in,
                       uint64_t ne, uint8_t* out) {
  for (uint64_t j = 0; j < ne; j++) {
    int64_t q;
    if (ts == 4) {
      float x;
      memcpy(&x, in + 4 * j, 4);
      q = (int64_t)roundf((x - (float)of) / (float)sc);
    } else {
      double x;
      memcpy(&x, in + 8 * j, 8);
      q = (int64_t)round((x - of) / sc);
    }
    st(out + bw * j, (uint64_t)q, bw);
  }
}

static void fscale_rev(uint32_t ts, uint32_t bw, double sc, double of, const uint8_t* in,
                       uint64_t ne, uint8_t* out) {
  for (uint64_t j = 0; j < ne; j++) {
    int64_t q = sext(ld(in + bw * j, bw), bw);
    if (ts == 4) {
      volatile double prod = sc * (double)(float)q;
      float y = (float)(prod + of);
      memcpy(out + 4 * j, &y, 4);
    } else {
      volatile double prod = sc * (double)q;
      double y = prod + of;
      memcpy(out + 8 * j, &y, 8);
    }
  }
}

static int is_compression_type(uint8_t t) {
  return t == TDBG_FILTER_GZIP || t == TDBG_FILTER_ZSTD || t == TDBG_FILTER_LZ4 ||
         t == TDBG_FILTER_RLE || t == TDBG_FILTER_BZIP2 ||
         t == TDBG_FILTER_DOUBLE_DELTA || t == TDBG_FILTER_DICTIONARY ||
         t == TDBG_FILTER_DELTA;
}

/* compressor_to_filter (compressor.h) */
static uint8_t compressor_filter_type(uint8_t c) {
  switch (c) {
    case TDBG_COMPRESSOR_NONE: return TDBG_FILTER_NONE;
    case TDBG_COMPRESSOR_GZIP: return TDBG_FILTER_GZIP;
    case TDBG_COMPRESSOR_ZSTD: return TDBG_FILTER_ZSTD;
    case TDBG_COMPRESSOR_LZ4: return TDBG_FILTER_LZ4;
    case TDBG_COMPRESSOR_RLE: return TDBG_FILTER_RLE;
    case TDBG_COMPRESSOR_BZIP2: return TDBG_FILTER_BZIP2;
    case TDBG_COMPRESSOR_DOUBLE_DELTA: return TDBG_FILTER_DOUBLE_DELTA;
    case TDBG_COMPRESSOR_DICTIONARY: return TDBG_FILTER_DICTIONARY;
    case TDBG_COMPRESSOR_DELTA: return TDBG_FILTER_DELTA;
    default: return 0xff;
  }
}

int oracle_pipeline_parse(const uint8_t* b, size_t len, uint32_t version,
                          uint8_t datatype, uint64_t cell_size,
                          oracle_pipeline* out, size_t* consumed) {
  size_t o = 0;
#define NEED(k) do { if (o + (k) > len) return TDBG_E_DESCRIPTOR; } while (0)
  if (!b || !out) return TDBG_E_ARG;
  memset(out, 0, sizeof(*out));
  NEED(8);
  out->max_chunk_size = (uint32_t)ld(b, 4);
  out->nfilters = (uint32_t)ld(b + 4, 4);
  o = 8;
  if (out->nfilters > ORACLE_MAX_FILTERS) return TDBG_E_DESCRIPTOR;
  out->version = version;
  out->on_disk_type = datatype;
  out->cell_size = cell_size;
  uint8_t cur = datatype;
  for (uint32_t i = 0; i < out->nfilters; i++) {
    oracle_filter* f = &out->f[i];
    NEED(5);
    uint8_t type = b[o];
    uint32_t mdlen = (uint32_t)ld(b + o + 1, 4);
    o += 5;
    /* filter_create.cc:109-113 */
    if (len - o < mdlen) return TDBG_E_DESCRIPTOR;
    f->reinterpret = TDBG_ANY;
    f->type = type;
    switch (type) {
      case TDBG_FILTER_NONE:
        break;
      case TDBG_FILTER_GZIP: case TDBG_FILTER_ZSTD: case TDBG_FILTER_LZ4:
      case TDBG_FILTER_RLE: case TDBG_FILTER_BZIP2: case TDBG_FILTER_DELTA:
      case TDBG_FILTER_DOUBLE_DELTA: case TDBG_FILTER_DICTIONARY: {
        NEED(5);
        f->compressor = b[o];
        f->level = (int32_t)ld(b + o + 1, 4);
        o += 5;
        if ((version >= 20 && type == TDBG_FILTER_DOUBLE_DELTA) ||
            (version >= 19 && type == TDBG_FILTER_DELTA)) {
          NEED(1);
          f->reinterpret = b[o];
          o += 1;
        }
        /* CompressionFilter(compressor,...) takes its type from the
         * compressor byte (compression_filter.cc:78-91). */
        f->type = compressor_filter_type(f->compressor);
        if (f->type == 0xff) return TDBG_E_DESCRIPTOR;
        break;
      }
      case TDBG_FILTER_BIT_WIDTH_REDUCTION:
      case TDBG_FILTER_POSITIVE_DELTA:
        NEED(4);
        f->window = (uint32_t)ld(b + o, 4);
        o += 4;
        break;
      case TDBG_FILTER_BITSHUFFLE: case TDBG_FILTER_BYTESHUFFLE:
      case TDBG_FILTER_AES_256_GCM: case TDBG_FILTER_CHECKSUM_MD5:
      case TDBG_FILTER_CHECKSUM_SHA256: case TDBG_FILTER_XOR:
        break;
      case TDBG_FILTER_SCALE_FLOAT: /* FilterConfig {double scale, offset; u64 byte_width} */
        NEED(24);
        memcpy(&f->scale, b + o, 8);
        memcpy(&f->offset, b + o + 8, 8);
        memcpy(&f->byte_width, b + o + 16, 8);
        o += 24;
        break;
      case TDBG_FILTER_WEBP:
        o += mdlen;
        break;
      default:
        return TDBG_E_DESCRIPTOR;
    }
    f->datatype = cur;
    cur = output_datatype(f, cur);
  }
  if (consumed) *consumed = o;
  return TDBG_OK;
#undef NEED
}

int oracle_pipeline_serialize(const oracle_pipeline* p, uint8_t* out,
                              size_t cap, size_t* len) {
  size_t o = 0;
#define PUT(v, w) do { if (o + (w) > cap) return TDBG_E_ARG; st(out + o, (uint64_t)(v), (w)); o += (w); } while (0)
  PUT(p->max_chunk_size, 4);
  PUT(p->nfilters, 4);
  for (uint32_t i = 0; i < p->nfilters; i++) {
    const oracle_filter* f = &p->f[i];
    /* filter.cc:100-112 + each serialize_impl */
    if (is_compression_type(f->type)) {
      int has_re = (f->type == TDBG_FILTER_DOUBLE_DELTA || f->type == TDBG_FILTER_DELTA);
      PUT(f->type, 1);
      PUT(has_re ? 6 : 5, 4);
      PUT(f->compressor, 1);
      PUT((uint32_t)f->level, 4);
      if (has_re) PUT(f->reinterpret, 1);
    } else if (f->type == TDBG_FILTER_BIT_WIDTH_REDUCTION ||
               f->type == TDBG_FILTER_POSITIVE_DELTA) {
      PUT(f->type, 1);
      PUT(4, 4);
      PUT(f->window, 4);
    } else if (f->type == TDBG_FILTER_NONE || f->type == TDBG_FILTER_BITSHUFFLE ||
               f->type == TDBG_FILTER_BYTESHUFFLE || f->type == TDBG_FILTER_XOR ||
               f->type == TDBG_FILTER_CHECKSUM_MD5 ||
               f->type == TDBG_FILTER_CHECKSUM_SHA256) {
      PUT(f->type, 1);
      PUT(0, 4);
    } else if (f->type == TDBG_FILTER_SCALE_FLOAT) {
      uint64_t sb, ob;
      memcpy(&sb, &f->scale, 8);
      memcpy(&ob, &f->offset, 8);
      PUT(f->type, 1);
      PUT(24, 4);
      PUT(sb, 8);
      PUT(ob, 8);
      PUT(f->byte_width, 8);
    } else {
      return TDBG_E_UNSUPPORTED;
    }
  }
  *len = o;
  return TDBG_OK;
#undef PUT
}

/* ------------------------------------------------------------------------ */
/* c-blosc2 shuffle / bitshuffle (generic semantics)                         */
/* ------------------------------------------------------------------------ */
/* shuffle_generic_inline / unshuffle_generic_inline: N = size/ts elements are
 * byte-transposed, the size%ts tail is copied. */
int oracle_byteshuffle(int inverse, uint32_t ts, const uint8_t* in, uint64_t n,
                       uint8_t* out) {
  if (ts == 0) return TDBG_E_ARG;
  uint64_t N = n / ts, r = n % ts;
  for (uint64_t j = 0; j < ts; j++)
    for (uint64_t i = 0; i < N; i++) {
      if (inverse) out[i * ts + j] = in[j * N + i];
      else out[j * N + i] = in[i * ts + j];
    }
  memcpy(out + (n - r), in + (n - r), r);
  return TDBG_OK;
}

/* One blosc2_bitshuffle / blosc2_bitunshuffle call on a block: the first
 * n8 = (n - n%8) elements are bit-transposed (kiyo-masui bshuf_trans_bit_elem),
 * the remaining bytes copied.  Bit plane p = 8*b + k holds bit k
 * of byte b of every element; element i's bit sits at bit i%8 of plane byte
 * i/8. */
int oracle_bitshuffle_block(int inverse, uint32_t ts, const uint8_t* in,
                            uint64_t nbytes, uint8_t* out) {
  if (ts == 0) return TDBG_E_ARG;
  uint64_t n = nbytes / ts;
  uint64_t n8 = n - n % 8;
  uint64_t rowb = n8 / 8; /* bytes per bit plane */
  if (!inverse) memset(out, 0, n8 * ts);
  else memset(out, 0, n8 * ts);
  for (uint64_t i = 0; i < n8; i++)
    for (uint32_t b = 0; b < ts; b++)
      for (uint32_t k = 0; k < 8; k++) {
        uint64_t plane = 8ull * b + k;
        uint64_t pbyte = plane * rowb + i / 8;
        if (!inverse) {
          uint32_t bit = (in[i * ts + b] >> k) & 1u;
          out[pbyte] |= (uint8_t)(bit << (i % 8));
        } else {
          uint32_t bit = (in[pbyte] >> (i % 8)) & 1u;
          out[i * ts + b] |= (uint8_t)(bit << k);
        }
      }
  memcpy(out + n8 * ts, in + n8 * ts, nbytes - n8 * ts);
  return TDBG_OK;
}

/* BitshuffleFilter::shuffle_part blocks of min(remaining, 8192) bytes,
 * bitshuffle_filter.cc:48,128-166. */
static void bitshuffle_part(int inverse, uint32_t ts, const uint8_t* in,
                            uint64_t n, uint8_t* out) {
  uint64_t done = 0;
  while (done < n) {
    uint64_t blk = n - done < 8192 ? n - done : 8192;
    oracle_bitshuffle_block(inverse, ts, in + done, blk, out + done);
    done += blk;
  }
}

/* ------------------------------------------------------------------------ */
/* RLE (rle_compressor.cc:51-141)                                            */
/* ------------------------------------------------------------------------ */
int oracle_rle_compress(uint64_t vs, const uint8_t* in, uint64_t n,
                        uint8_t* out, uint64_t cap, uint64_t* out_len) {
  uint64_t o = 0;
  if (!in) return TDBG_E_ARG;
  if (vs == 0) return TDBG_E_ARG;
  uint64_t nv = n / vs;
  *out_len = 0;
  if (nv == 0) return TDBG_OK; /* :64-66 */
  if (n % vs) return TDBG_E_RLE_FORMAT; /* :68-71 */
  uint32_t run = 1;
  const uint8_t* prev = in;
  const uint8_t* cur = in + vs;
  for (uint64_t i = 1; i < nv; i++) {
    if (memcmp(cur, prev, vs) == 0 && run < 65535) {
      run++;
    } else {
      if (o + vs + 2 > cap) return TDBG_E_OUT_FULL;
      memcpy(out + o, prev, vs);
      out[o + vs] = (uint8_t)(run >> 8);
      out[o + vs + 1] = (uint8_t)(run % 256);
      o += vs + 2;
      run = 1;
    }
    prev = cur;
    cur = prev + vs;
  }
  if (o + vs + 2 > cap) return TDBG_E_OUT_FULL;
  memcpy(out + o, prev, vs);
  out[o + vs] = (uint8_t)(run >> 8);
  out[o + vs + 1] = (uint8_t)(run % 256);
  o += vs + 2;
  *out_len = o;
  return TDBG_OK;
}

/* Returns status; *written = bytes written to out. */
static int rle_decompress_w(uint64_t vs, const uint8_t* in, uint64_t n,
                            uint8_t* out, uint64_t out_size,
                            uint64_t* written) {
  uint64_t rs = vs + 2;
  uint64_t nr = n / rs;
  uint64_t o = 0;
  *written = 0;
  if (nr == 0) return TDBG_OK; /* :115-117 */
  if (n % rs) return TDBG_E_RLE_FORMAT; /* :119-123 */
  for (uint64_t i = 0; i < nr; i++) {
    const uint8_t* r = in + i * rs;
    uint64_t len = ((uint64_t)r[vs] << 8) + r[vs + 1];
    for (uint64_t j = 0; j < len; j++) {
      if (o + vs > out_size) { *written = o; return TDBG_E_OUT_FULL; }
      memcpy(out + o, r, vs);
      o += vs;
    }
  }
  *written = o;
  return TDBG_OK;
}

int oracle_rle_decompress(uint64_t vs, const uint8_t* in, uint64_t n,
                          uint8_t* out, uint64_t out_size) {
  uint64_t w;
  if (!in) return TDBG_E_ARG;
  return rle_decompress_w(vs, in, n, out, out_size, &w);
}

/* ------------------------------------------------------------------------ */
/* Double delta (dd_compressor.cc:211-450, format_spec/filters/double_delta.md) */
/* ------------------------------------------------------------------------ */
/* checked arithmetic (tiledb/common/arithmetic.h:89-264) collapsed: deltas
 * are computed in the "extended" type: int64 for signed T, and for unsigned
 * T either int64 (<= 32-bit, which never overflows) or the uint64
 * sub_signed rule. */
static int dd_delta(uint64_t cur, uint64_t prev, const ival_t* t, int64_t* d) {
  if (t->sgn || t->w < 8) {
    if (t->w < 8) {
      int64_t a = t->sgn ? sext(cur, t->w) : (int64_t)cur;
      int64_t b = t->sgn ? sext(prev, t->w) : (int64_t)prev;
      *d = a - b;
      return TDBG_OK;
    }
    /* checked_arithmetic<int64_t>::sub */
    int64_t a = (int64_t)cur, b = (int64_t)prev;
    if (__builtin_sub_overflow(a, b, d)) return TDBG_E_DD_OVERFLOW;
    return TDBG_OK;
  }
  /* checked_arithmetic<uint64_t>::sub_signed */
  if (cur >= prev) {
    uint64_t r = cur - prev;
    if (r > (uint64_t)INT64_MAX) return TDBG_E_DD_OVERFLOW;
    *d = (int64_t)r;
    return TDBG_OK;
  }
  uint64_t r = prev - cur;
  if (r > (uint64_t)INT64_MAX) {
    if (r == (uint64_t)INT64_MAX + 1) { *d = INT64_MIN; return TDBG_OK; }
    return TDBG_E_DD_OVERFLOW;
  }
  *d = -(int64_t)r;
  return TDBG_OK;
}

/* checked_arithmetic<int64_t>::sub with its min-value special case. */
static int chk_sub64(int64_t a, int64_t b, int64_t* r) {
  if (__builtin_sub_overflow(a, b, r)) return TDBG_E_DD_OVERFLOW;
  return TDBG_OK;
}

static uint64_t uabs64(int64_t v) { return v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v; }

int oracle_dd_compress(uint8_t dtype, const uint8_t* in, uint64_t n,
                       uint8_t* out, uint64_t cap, uint64_t* out_len) {
  ival_t t;
  int rc = dd_type(dtype, &t);
  if (rc) return rc;
  uint64_t num = n / t.w;
  if (num == 0) return TDBG_E_ARG; /* iassert(num > 0) dd_compressor.cc:216 */
  /* compute_bitsize :267-303 (first delta counts) */
  uint32_t bitsize = 0;
  if (num > 2) {
    uint64_t maxd = 0;
    int64_t prevd = 0;
    for (uint64_t i = 1; i < num; i++) {
      int64_t d;
      rc = dd_delta(ld(in + i * t.w, t.w), ld(in + (i - 1) * t.w, t.w), &t, &d);
      if (rc) return rc;
      if (i > 1) {
        int64_t dd;
        rc = chk_sub64(d, prevd, &dd);
        if (rc) return rc;
        uint64_t a = uabs64(dd);
        if (a > maxd) maxd = a;
      } else {
        maxd = uabs64(d);
      }
      prevd = d;
    }
    do { ++bitsize; maxd >>= 1; } while (maxd);
  }
  uint64_t o = 0;
#define WR(src, k) do { if (o + (k) > cap) return TDBG_E_OUT_FULL; memcpy(out + o, (src), (k)); o += (k); } while (0)
  uint8_t bc = (uint8_t)bitsize;
  WR(&bc, 1);
  WR(&num, 8);
  if (bitsize >= t.w * 8 - 1) { /* :233-236 raw */
    WR(in, n);
    *out_len = o;
    return TDBG_OK;
  }
  WR(in, t.w);
  if (num == 1) { *out_len = o; return TDBG_OK; }
  WR(in + t.w, t.w);
  if (num == 2) { *out_len = o; return TDBG_OK; }
  /* :249-261 double deltas, each [sign][bitsize bits], MSB-first in u64 */
  int64_t prevd = (int64_t)((uint64_t)(t.sgn ? sext(ld(in + t.w, t.w), t.w) : (int64_t)ld(in + t.w, t.w)) -
                             (uint64_t)(t.sgn ? sext(ld(in, t.w), t.w) : (int64_t)ld(in, t.w)));
  uint64_t chunk = 0;
  int bit = 63;
  for (uint64_t i = 2; i < num; i++) {
    int64_t a = t.sgn ? sext(ld(in + i * t.w, t.w), t.w) : (int64_t)ld(in + i * t.w, t.w);
    int64_t b = t.sgn ? sext(ld(in + (i - 1) * t.w, t.w), t.w) : (int64_t)ld(in + (i - 1) * t.w, t.w);
    int64_t curd = (int64_t)((uint64_t)a - (uint64_t)b);
    int64_t dd = (int64_t)((uint64_t)curd - (uint64_t)prevd);
    /* write_double_delta :406-450 */
    uint64_t code_sign = dd < 0 ? 1 : 0;
    uint64_t mag = uabs64(dd);
    for (int k = (int)bitsize; k >= 0; k--) {
      uint64_t bitv = (k == (int)bitsize) ? code_sign : ((mag >> k) & 1ull);
      chunk |= bitv << bit;
      if (--bit < 0) { WR(&chunk, 8); chunk = 0; bit = 63; }
    }
    prevd = curd;
  }
  if (bit < 63) WR(&chunk, 8);
  *out_len = o;
  return TDBG_OK;
#undef WR
}

/* DoubleDelta::decompress :314-404.  *written receives bytes written. */
static int dd_decompress_w(uint8_t dtype, const uint8_t* in, uint64_t n,
                           uint8_t* out, uint64_t out_size, uint64_t* written) {
  ival_t t;
  *written = 0;
  int rc = dd_type(dtype, &t);
  if (rc) return rc;
  uint64_t ip = 0, op = 0;
#define RD(dst, k) do { if (ip + (k) > n) return TDBG_E_DATA_READ; memcpy((dst), in + ip, (k)); ip += (k); } while (0)
#define WRO(src, k) do { if (op + (k) > out_size) return TDBG_E_OUT_FULL; memcpy(out + op, (src), (k)); op += (k); *written = op; } while (0)
  uint8_t bc = 0;
  uint64_t num = 0;
  RD(&bc, 1);
  RD(&num, 8);
  uint32_t bitsize = bc;
  if (bitsize >= t.w * 8 - 1) {
    WRO(in + ip, n - ip);
    return TDBG_OK;
  }
  uint64_t v = 0;
  RD(&v, t.w);
  WRO(&v, t.w);
  if (num == 1) return TDBG_OK;
  RD(&v, t.w);
  WRO(&v, t.w);
  if (num == 2) return TDBG_OK;
  uint64_t chunk;
  RD(&chunk, 8);
  int bic = 63;
  for (uint64_t i = 2; i < num; i++) {
    /* read_double_delta :356-404 */
    int sign = ((chunk >> bic) & 1ull) ? -1 : 1;
    --bic;
    if (bic < 0) { RD(&chunk, 8); bic = 63; }
    int left = (int)bitsize;
    int take = bic + 1 < left ? bic + 1 : left;
    int bit_in_dd = (int)bitsize - 1;
    int64_t dd = 0;
    while (left > 0) {
      if (take > 0) {
        uint64_t tmp = ((chunk << (63 - bic)) >> (63 - bit_in_dd));
        dd |= (int64_t)tmp;
        bit_in_dd -= take;
        bic -= take;
        left -= take;
      }
      if (bic < 0 && ip != n) {
        RD(&chunk, 8);
        bic = 63;
        take = bic + 1 < left ? bic + 1 : left;
      }
      if (bic < 0 && left > 0 && ip == n) return TDBG_E_DATA_READ;
    }
    dd *= sign;
    uint64_t x1 = ld(out + (i - 1) * t.w, t.w), x2 = ld(out + (i - 2) * t.w, t.w);
    int64_t a = t.sgn ? sext(x1, t.w) : (int64_t)x1;
    int64_t b = t.sgn ? sext(x2, t.w) : (int64_t)x2;
    uint64_t val = (uint64_t)dd + 2 * (uint64_t)a - (uint64_t)b;
    val &= mask_w(t.w);
    WRO(&val, t.w);
  }
  return TDBG_OK;
#undef RD
#undef WRO
}

int oracle_dd_decompress(uint8_t dtype, const uint8_t* in, uint64_t n,
                         uint8_t* out, uint64_t out_size) {
  uint64_t w;
  return dd_decompress_w(dtype, in, n, out, out_size, &w);
}

/* Delta::compress / decompress (delta_compressor.cc:224-249, 251-273); the
 * value type table is DoubleDelta's (dd_type; delta_compressor.cc:60-217).
 * Forward: [u64 num][T x0][T (x[i] - x[i-1])]..., the difference truncated
 * to T (wrapping).  Reverse: x[i] = (T)(x[i-1] + d[i]); x0 is read and
 * written even when num == 0.  Reads fail before the write at the same index
 * (DATA_READ), writes past the part's size fail with OUT_FULL.  Bytes past
 * the decoded values are unspecified in the reference; zero here. */
static int delta_compress(uint8_t dtype, const uint8_t* in, uint64_t n,
                          uint8_t* out, uint64_t cap, uint64_t* out_n) {
  ival_t t;
  int rc = dd_type(dtype, &t);
  if (rc) return rc == TDBG_E_DD_TYPE ? TDBG_E_DELTA_TYPE : rc; /* :210-213 */
  uint64_t num = n / t.w;
  if (cap < 8 + (num ? num : 1) * t.w) return TDBG_E_ARG;
  memcpy(out, &num, 8);
  st(out + 8, num ? ld(in, t.w) : 0, t.w);
  for (uint64_t i = 1; i < num; i++)
    st(out + 8 + i * t.w, (ld(in + i * t.w, t.w) - ld(in + (i - 1) * t.w, t.w)) & mask_w(t.w), t.w);
  *out_n = 8 + (num ? num : 1) * t.w;
  return TDBG_OK;
}

static int delta_decompress_w(uint8_t dtype, const uint8_t* in, uint64_t n,
                              uint8_t* out, uint64_t out_size, uint64_t* written) {
  ival_t t;
  *written = 0;
  int rc = dd_type(dtype, &t);
  if (rc) return rc == TDBG_E_DD_TYPE ? TDBG_E_DELTA_TYPE : rc; /* :210-213 */
  uint64_t num = 0;
  if (n < 8) return TDBG_E_DATA_READ;
  memcpy(&num, in, 8);
  uint64_t nv = num ? num : 1, prev = 0;
  for (uint64_t i = 0; i < nv; i++) {
    if (8 + (i + 1) * t.w > n) return TDBG_E_DATA_READ;
    if ((i + 1) * t.w > out_size) return TDBG_E_OUT_FULL;
    uint64_t d = ld(in + 8 + i * t.w, t.w);
    prev = i == 0 ? d : (prev + d) & mask_w(t.w);
    st(out + i * t.w, prev, t.w);
    *written = (i + 1) * t.w;
  }
  if (*written < out_size) memset(out + *written, 0, out_size - *written);
  return TDBG_OK;
}

/* ------------------------------------------------------------------------ */
/* Forward pipeline (fixture producer)                                       */
/* ------------------------------------------------------------------------ */
#define MAXPARTS 96
typedef struct { const uint8_t* p; uint64_t n; } part_t;
typedef struct { part_t v[MAXPARTS]; int np; } plist_t;
typedef struct { void* blocks[4 * ORACLE_MAX_FILTERS + 8]; int nb; } arena_t;

static uint8_t* arena_alloc(arena_t* a, uint64_t n) {
  if (a->nb >= (int)(sizeof(a->blocks) / sizeof(a->blocks[0]))) return NULL;
  uint8_t* p = (uint8_t*)calloc(1, n ? n : 1);
  a->blocks[a->nb++] = p;
  return p;
}
static void arena_free(arena_t* a) {
  for (int i = 0; i < a->nb; i++) free(a->blocks[i]);
  a->nb = 0;
}
static uint64_t plist_size(const plist_t* l) {
  uint64_t s = 0;
  for (int i = 0; i < l->np; i++) s += l->v[i].n;
  return s;
}
static int plist_push(plist_t* l, const uint8_t* p, uint64_t n) {
  if (n == 0) return TDBG_OK; /* empty views are skipped, filter_buffer.cc:511 */
  if (l->np >= MAXPARTS) return TDBG_E_UNSUPPORTED;
  l->v[l->np].p = p;
  l->v[l->np].n = n;
  l->np++;
  return TDBG_OK;
}
/* out_md = [hdr] + in_md (prepend after append_view) */
static int md_prepend(plist_t* out, const uint8_t* hdr, uint64_t n, const plist_t* in) {
  out->np = 0;
  int rc = plist_push(out, hdr, n);
  if (rc) return rc;
  for (int i = 0; i < in->np; i++) {
    rc = plist_push(out, in->v[i].p, in->v[i].n);
    if (rc) return rc;
  }
  return TDBG_OK;
}

static int fwd_filter(const oracle_pipeline* p, const oracle_filter* f,
                      const plist_t* D, const plist_t* M, plist_t* D2,
                      plist_t* M2, arena_t* ar) {
  int rc;
  uint64_t dsize = plist_size(D);
  D2->np = 0;
  M2->np = 0;
  switch (f->type) {
    case TDBG_FILTER_NONE:
      *D2 = *D; *M2 = *M;
      return TDBG_OK;
    case TDBG_FILTER_BYTESHUFFLE: { /* byteshuffle_filter.cc:60-89 */
      uint32_t ts = (uint32_t)oracle_datatype_size(f->datatype);
      uint8_t* out = arena_alloc(ar, dsize);
      uint8_t* hdr = arena_alloc(ar, 4 + 4 * (uint64_t)D->np);
      if (!out || !hdr) return TDBG_E_ARG;
      st(hdr, (uint64_t)D->np, 4);
      uint64_t o = 0;
      for (int i = 0; i < D->np; i++) {
        st(hdr + 4 + 4 * i, D->v[i].n, 4);
        oracle_byteshuffle(0, ts, D->v[i].p, D->v[i].n, out + o);
        o += D->v[i].n;
      }
      plist_push(D2, out, dsize);
      return md_prepend(M2, hdr, 4 + 4 * (uint64_t)D->np, M);
    }
    case TDBG_FILTER_SCALE_FLOAT: { /* float_scaling_filter.cc:60-99 */
      uint32_t ts = (uint32_t)oracle_datatype_size(f->datatype), bw = (uint32_t)f->byte_width;
      if ((ts != 4 && ts != 8) || (bw != 1 && bw != 2 && bw != 4 && bw != 8)) return TDBG_E_ARG;
      uint64_t tot = 0;
      for (int i = 0; i < D->np; i++) tot += D->v[i].n / ts * bw;
      uint8_t* out = arena_alloc(ar, tot ? tot : 1);
      uint8_t* hdr = arena_alloc(ar, 4 + 4 * (uint64_t)D->np);
      if (!out || !hdr) return TDBG_E_ARG;
      st(hdr, (uint64_t)D->np, 4);
      uint64_t o = 0;
      for (int i = 0; i < D->np; i++) {
        uint64_t ne = D->v[i].n / ts;
        st(hdr + 4 + 4 * i, ne * bw, 4);
        fscale_fwd(ts, bw, f->scale, f->offset, D->v[i].p, ne, out + o);
        o += ne * bw;
      }
      plist_push(D2, out, tot);
      return md_prepend(M2, hdr, 4 + 4 * (uint64_t)D->np, M);
    }
    case TDBG_FILTER_XOR: { /* xor_filter.cc:120-146: one part per input buffer */
      uint32_t ts = (uint32_t)oracle_datatype_size(f->datatype);
      if (ts != 1 && ts != 2 && ts != 4 && ts != 8) return TDBG_E_ARG;
      uint8_t* out = arena_alloc(ar, dsize);
      uint8_t* hdr = arena_alloc(ar, 4 + 4 * (uint64_t)D->np);
      if (!out || !hdr) return TDBG_E_ARG;
      memset(out, 0, dsize);
      st(hdr, (uint64_t)D->np, 4);
      uint64_t o = 0;
      for (int i = 0; i < D->np; i++) {
        st(hdr + 4 + 4 * i, D->v[i].n, 4);
        xor_part(0, ts, D->v[i].p, D->v[i].n, out + o);
        o += D->v[i].n;
      }
      plist_push(D2, out, dsize);
      return md_prepend(M2, hdr, 4 + 4 * (uint64_t)D->np, M);
    }
    case TDBG_FILTER_BITSHUFFLE: { /* bitshuffle_filter.cc:63-126 */
      uint32_t ts = (uint32_t)oracle_datatype_size(f->datatype);
      plist_t parts = {0};
      for (int i = 0; i < D->np; i++) {
        uint64_t n = D->v[i].n, rem = n % 8;
        if (rem == 0) plist_push(&parts, D->v[i].p, n);
        else {
          plist_push(&parts, D->v[i].p, n - rem);
          plist_push(&parts, D->v[i].p + n - rem, rem);
        }
      }
      uint8_t* out = arena_alloc(ar, dsize);
      uint8_t* hdr = arena_alloc(ar, 4 + 4 * (uint64_t)parts.np);
      if (!out || !hdr) return TDBG_E_ARG;
      st(hdr, (uint64_t)parts.np, 4);
      uint64_t o = 0;
      for (int i = 0; i < parts.np; i++) {
        uint64_t n = parts.v[i].n;
        st(hdr + 4 + 4 * i, n, 4);
        if (n % ts != 0 || n % 8 != 0) memcpy(out + o, parts.v[i].p, n);
        else bitshuffle_part(0, ts, parts.v[i].p, n, out + o);
        o += n;
      }
      plist_push(D2, out, dsize);
      return md_prepend(M2, hdr, 4 + 4 * (uint64_t)parts.np, M);
    }
    case TDBG_FILTER_BIT_WIDTH_REDUCTION: { /* bwr.cc:110-280 */
      ival_t t = bwr_type(f->datatype, p->version);
      if (!t.active) { *D2 = *D; *M2 = *M; return TDBG_OK; }
      uint32_t w = t.w;
      uint64_t total_win = 0;
      for (int i = 0; i < D->np; i++) {
        uint32_t ps = (uint32_t)D->v[i].n;
        uint32_t ws = (ps < f->window ? ps : f->window) / w * w;
        if (ws == 0) return TDBG_E_ARG; /* division by zero in the reference */
        total_win += ps / ws + (ps % ws ? 1 : 0);
      }
      uint8_t* out = arena_alloc(ar, dsize);
      uint64_t mdn = 8 + total_win * (4 + w + 1);
      uint8_t* hdr = arena_alloc(ar, mdn);
      if (!out || !hdr) return TDBG_E_ARG;
      st(hdr, dsize, 4);
      st(hdr + 4, total_win, 4);
      uint64_t mo = 8, o = 0;
      for (int i = 0; i < D->np; i++) {
        const uint8_t* in = D->v[i].p;
        uint32_t ps = (uint32_t)D->v[i].n;
        uint32_t ws = (ps < f->window ? ps : f->window) / w * w;
        uint32_t nw = ps / ws + (ps % ws ? 1 : 0);
        uint64_t ip = 0;
        for (uint32_t k = 0; k < nw; k++) {
          uint32_t nb = ws < ps - k * ws ? ws : ps - k * ws;
          uint32_t ne = nb / w;
          /* compute_bits_required :406-447 */
          uint8_t bits = (uint8_t)(8 * w);
          uint64_t minv = 0;
          {
            int have = 0;
            if (t.sgn) {
              int64_t mn = 0, mx = 0;
              for (uint32_t j = 0; j < ne; j++) {
                int64_t v = sext(ld(in + ip + (uint64_t)j * w, w), w);
                if (!have || v < mn) mn = v;
                if (!have || v > mx) mx = v;
                have = 1;
              }
              if (have) {
                /* checked sub/add in the extended type */
                int ovf = 0;
                int64_t range = 0;
                if (w < 8) {
                  range = mx - mn;
                  int64_t lim = (int64_t)(mask_w(w) >> 1);
                  if (range > lim || range + 1 > lim) ovf = 1;
                } else {
                  if (__builtin_sub_overflow(mx, mn, &range)) ovf = 1;
                  else if (range == INT64_MAX) ovf = 1;
                }
                if (!ovf) {
                  int64_t ro = range + 1;
                  bits = ro <= 127 ? 8 : ro <= 32767 ? 16 : ro <= 2147483647LL ? 32 : 64;
                  minv = (uint64_t)mn;
                }
              }
            } else {
              uint64_t mn = 0, mx = 0;
              for (uint32_t j = 0; j < ne; j++) {
                uint64_t v = ld(in + ip + (uint64_t)j * w, w);
                if (!have || v < mn) mn = v;
                if (!have || v > mx) mx = v;
                have = 1;
              }
              if (have) {
                uint64_t range = mx - mn;
                if (range != mask_w(w)) { /* range + 1 overflows T */
                  uint64_t ro = range + 1;
                  uint32_t nbits = 0;
                  while (ro) { nbits++; ro >>= 1; }
                  bits = nbits <= 8 ? 8 : nbits <= 16 ? 16 : nbits <= 32 ? 32 : 64;
                  minv = mn;
                }
              }
            }
          }
          /* window header [T offset][u8 bits][u32 nbytes]; the offset of an
           * overflowing window is left uninitialized by the reference
           * (:421-430) -- written as 0 here. */
          st(hdr + mo, minv, w);
          hdr[mo + w] = bits;
          st(hdr + mo + w + 1, nb, 4);
          mo += w + 5;
          if (bits >= 8 * w || nb % w != 0) {
            memcpy(out + o, in + ip, nb);
            o += nb;
            ip += nb;
          } else {
            uint32_t cb = bits / 8;
            for (uint32_t j = 0; j < ne; j++) {
              uint64_t rel = (ld(in + ip, w) - minv) & mask_w(w);
              st(out + o, rel, cb);
              o += cb;
              ip += w;
            }
          }
        }
      }
      plist_push(D2, out, o);
      return md_prepend(M2, hdr, mdn, M);
    }
    case TDBG_FILTER_POSITIVE_DELTA: { /* pd.cc:140-245 */
      ival_t t = pd_type(f->datatype, p->version);
      if (!t.active) { *D2 = *D; *M2 = *M; return TDBG_OK; }
      uint32_t w = t.w;
      uint64_t total_win = 0;
      for (int i = 0; i < D->np; i++) {
        uint32_t ps = (uint32_t)D->v[i].n;
        uint32_t ws = (ps < f->window ? ps : f->window) / w * w;
        if (ws == 0) return TDBG_E_ARG;
        total_win += ps / ws + (ps % ws ? 1 : 0);
      }
      uint8_t* out = arena_alloc(ar, dsize);
      uint64_t mdn = 4 + total_win * (4 + w);
      uint8_t* hdr = arena_alloc(ar, mdn);
      if (!out || !hdr) return TDBG_E_ARG;
      st(hdr, total_win, 4);
      uint64_t mo = 4, o = 0;
      for (int i = 0; i < D->np; i++) {
        const uint8_t* in = D->v[i].p;
        uint32_t ps = (uint32_t)D->v[i].n;
        uint32_t ws = (ps < f->window ? ps : f->window) / w * w;
        uint32_t nw = ps / ws + (ps % ws ? 1 : 0);
        uint64_t ip = 0;
        for (uint32_t k = 0; k < nw; k++) {
          uint32_t nb = ws < ps - k * ws ? ws : ps - k * ws;
          /* value<T>() reads past the end of a short last window (:217);
           * the bytes it would see are unspecified -- zero-filled here. */
          uint64_t first = 0;
          memcpy(&first, in + ip, (ps - ip) < w ? (ps - ip) : w);
          st(hdr + mo, first, w);
          st(hdr + mo + w, nb, 4);
          mo += w + 4;
          if (nb % w != 0) {
            memcpy(out + o, in + ip, nb);
            o += nb;
            ip += nb;
          } else {
            uint64_t prev = ld(in + ip, w);
            for (uint32_t j = 0; j < nb / w; j++) {
              uint64_t cur = ld(in + ip, w);
              int lt = t.sgn ? (sext(cur, w) < sext(prev, w)) : (cur < prev);
              if (lt) return TDBG_E_PD_DECREASING;
              st(out + o, (cur - prev) & mask_w(w), w);
              o += w;
              ip += w;
              prev = cur;
            }
          }
        }
      }
      plist_push(D2, out, o);
      return md_prepend(M2, hdr, mdn, M);
    }
    case TDBG_FILTER_RLE:
    case TDBG_FILTER_DELTA:
    case TDBG_FILTER_DOUBLE_DELTA: { /* compression_filter.cc:240-301 */
      plist_t parts = {0};
      for (int i = 0; i < M->np; i++) plist_push(&parts, M->v[i].p, M->v[i].n);
      int nmd = parts.np;
      for (int i = 0; i < D->np; i++) plist_push(&parts, D->v[i].p, D->v[i].n);
      int ndata = parts.np - nmd;
      uint64_t ub = 0;
      for (int i = 0; i < parts.np; i++)
        ub += parts.v[i].n + (f->type == TDBG_FILTER_RLE ? (parts.v[i].n / p->cell_size) * 2 : 17);
      uint8_t* out = arena_alloc(ar, ub + 64);
      uint64_t mdn = 8 + 8 * (uint64_t)parts.np;
      uint8_t* hdr = arena_alloc(ar, mdn);
      if (!out || !hdr) return TDBG_E_ARG;
      st(hdr, (uint64_t)nmd, 4);
      st(hdr + 4, (uint64_t)ndata, 4);
      uint64_t o = 0;
      uint8_t ddt = f->reinterpret != TDBG_ANY ? f->reinterpret : f->datatype;
      for (int i = 0; i < parts.np; i++) {
        uint64_t cl = 0;
        if (f->type == TDBG_FILTER_RLE)
          rc = oracle_rle_compress(p->cell_size, parts.v[i].p, parts.v[i].n, out + o, ub + 64 - o, &cl);
        else if (f->type == TDBG_FILTER_DELTA)
          rc = delta_compress(ddt, parts.v[i].p, parts.v[i].n, out + o, ub + 64 - o, &cl);
        else
          rc = oracle_dd_compress(ddt, parts.v[i].p, parts.v[i].n, out + o, ub + 64 - o, &cl);
        if (rc) return rc;
        st(hdr + 8 + 8 * i, parts.v[i].n, 4);
        st(hdr + 12 + 8 * i, cl, 4);
        o += cl;
      }
      plist_push(D2, out, o);
      M2->np = 0;
      return plist_push(M2, hdr, mdn);
    }
    default:
      if (is_compression_type(f->type) && f->compressor == TDBG_COMPRESSOR_NONE) {
        *D2 = *D; *M2 = *M; return TDBG_OK;
      }
      return TDBG_E_UNSUPPORTED;
  }
}

uint32_t oracle_compute_chunk_size(uint64_t tile_size, uint64_t cell_size,
                                   uint64_t max_chunk) {
  uint64_t mc = max_chunk ? max_chunk : 65536;
  uint64_t c = mc < tile_size ? mc : tile_size;
  c = c / cell_size * cell_size;
  if (c < cell_size) c = cell_size;
  return (uint32_t)c;
}

uint64_t oracle_filtered_bound(const oracle_pipeline* p, uint64_t size,
                               uint64_t max_chunk) {
  uint64_t cs = oracle_compute_chunk_size(size, p->cell_size ? p->cell_size : 1, max_chunk);
  uint64_t nch = size / (cs ? cs : 1) + 2;
  /* generous: data may grow by RLE (x3 worst) plus per-filter headers */
  return 8 + nch * (12 + 64 * 1024) + size * 4 + 4096;
}

int oracle_filter_tile(const oracle_pipeline* p, const uint8_t* tile,
                       uint64_t size, const uint64_t* offsets,
                       uint64_t noffsets, uint64_t max_chunk, uint8_t* out,
                       uint64_t cap, uint64_t* out_len) {
  uint64_t cell = p->cell_size ? p->cell_size : 1;
  uint32_t chunk = oracle_compute_chunk_size(size, cell, max_chunk);
  /* chunk boundaries: filter_pipeline.cc:151-230 */
  uint64_t nchunks = 1, last = chunk;
  uint64_t* coff = NULL;
  int var = offsets != NULL && noffsets > 0;
  if (var) {
    coff = (uint64_t*)malloc(sizeof(uint64_t) * (noffsets + 2));
    uint64_t nco = 0, cur = 0, mn = chunk / 2, mx = chunk + chunk / 2;
    coff[nco++] = 0;
    for (uint64_t c = 0; c < noffsets; c++) {
      uint64_t cs = c == noffsets - 1 ? size - offsets[c] : offsets[c + 1] - offsets[c];
      uint64_t ns = cur + cs;
      if (ns > chunk) {
        if (cur <= mn || ns <= mx) {
          coff[nco++] = offsets[c] + cs;
          cur = 0;
        } else {
          coff[nco++] = offsets[c];
          if (cs > chunk) {
            if (c != noffsets - 1) coff[nco++] = offsets[c] + cs;
            cur = 0;
          } else {
            cur = cs;
          }
        }
      } else {
        cur += cs;
      }
    }
    if (size != chunk) {
      nchunks = nco;
      last = size - coff[nchunks - 1];
    }
  } else if (size != chunk) {
    nchunks = size / chunk;
    last = size % chunk;
    if (last != 0) nchunks++;
    else last = chunk;
  }
  uint64_t o = 8;
  if (cap < 8) { free(coff); return TDBG_E_OUT_FULL; }
  st(out, nchunks, 8);
  int rc = TDBG_OK;
  for (uint64_t i = 0; i < nchunks && rc == TDBG_OK; i++) {
    uint64_t off = var ? coff[i] : i * chunk;
    uint64_t n = i == nchunks - 1 ? last : (var ? coff[i + 1] - coff[i] : chunk);
    arena_t ar = {{0}, 0};
    plist_t D = {0}, M = {0}, D2, M2;
    D.v[0].p = tile + off;
    D.v[0].n = n;
    D.np = 1;
    for (uint32_t k = 0; k < p->nfilters && rc == TDBG_OK; k++) {
      rc = fwd_filter(p, &p->f[k], &D, &M, &D2, &M2, &ar);
      D = D2;
      M = M2;
    }
    if (rc == TDBG_OK) {
      uint64_t ds = plist_size(&D), ms = plist_size(&M);
      if (o + 12 + ds + ms > cap) rc = TDBG_E_OUT_FULL;
      else {
        st(out + o, n, 4);
        st(out + o + 4, ds, 4);
        st(out + o + 8, ms, 4);
        o += 12;
        for (int k = 0; k < M.np; k++) { memcpy(out + o, M.v[k].p, M.v[k].n); o += M.v[k].n; }
        for (int k = 0; k < D.np; k++) { memcpy(out + o, D.v[k].p, D.v[k].n); o += D.v[k].n; }
      }
    }
    arena_free(&ar);
  }
  free(coff);
  *out_len = o;
  return rc;
}

/* ------------------------------------------------------------------------ */
/* Reverse pipeline (the checker)                                            */
/* ------------------------------------------------------------------------ */
/* FilterBuffer semantics collapsed to one contiguous buffer per stage (in
 * reverse every stage has exactly one data buffer and one md stream). */
typedef struct {
  uint8_t* p;
  uint64_t cap;  /* prepend_buffer size / fixed allocation size   */
  uint64_t size; /* FilterBuffer::size(): written bytes, or cap if fixed */
  int fixed;
  int owned;
} obuf_t;

typedef struct { const uint8_t* p; uint64_t n, off; } mdcur_t;

static int md_read(mdcur_t* c, void* dst, uint64_t k) {
  if (c->off + k > c->n) return TDBG_E_MD_READ;
  memcpy(dst, c->p + c->off, k);
  c->off += k;
  return TDBG_OK;
}

/* prepend_buffer(nbytes) on the output (filter_buffer.cc:472-506). */
static int out_prepend(obuf_t* o, uint64_t nbytes) {
  if (o->fixed) return nbytes > o->cap ? TDBG_E_OUT_FULL : TDBG_OK;
  o->p = (uint8_t*)calloc(1, nbytes ? nbytes : 1);
  o->cap = nbytes;
  o->size = 0;
  o->owned = 1;
  return TDBG_OK;
}

/* FilterBuffer::write(FilterBuffer* other, n) from input position ip
 * (filter_buffer.cc:393-424): copies the available input, failing on a full
 * output first, then on a short input. */
static int copy_in_out(const uint8_t* in, uint64_t in_n, uint64_t ip,
                       obuf_t* o, uint64_t* op, uint64_t n) {
  uint64_t avail = ip < in_n ? in_n - ip : 0;
  uint64_t k = n < avail ? n : avail;
  uint64_t room = o->cap - *op;
  if (k > 0 && room == 0) return TDBG_E_OUT_FULL;
  if (k > room) {
    memcpy(o->p + *op, in + ip, room);
    *op += room;
    return TDBG_E_OUT_FULL;
  }
  memcpy(o->p + *op, in + ip, k);
  *op += k;
  if (k < n) return TDBG_E_DATA_READ;
  return TDBG_OK;
}

static void finish_size(obuf_t* o, uint64_t op) {
  if (!o->fixed) o->size = op;
  else o->size = o->cap;
}

static int rev_filter(const oracle_pipeline* p, const oracle_filter* f,
                      const uint8_t* in, uint64_t in_n, mdcur_t* md,
                      obuf_t* out, uint8_t** newmd, uint64_t* newmd_n,
                      int* md_replaced) {
  int rc;
  *md_replaced = 0;
  /* pass-through: append_view(input) (e.g. bwr.cc:339-349) */
#define PASS_THROUGH()                                                  \
  do {                                                                  \
    if (out->fixed) {                                                   \
      if (in_n > out->cap) return TDBG_E_OUT_FULL;                      \
      memcpy(out->p, in, in_n);                                         \
      out->size = out->cap;                                             \
    } else {                                                            \
      out->p = (uint8_t*)in; out->cap = in_n; out->size = in_n; out->owned = 0; \
    }                                                                   \
    return TDBG_OK;                                                     \
  } while (0)

  switch (f->type) {
    case TDBG_FILTER_NONE:
      PASS_THROUGH();
    case TDBG_FILTER_SCALE_FLOAT: {
      /* float_scaling_filter.cc:164-197, 217-238: one output prepend per
       * part; a fixed allocation allows only the first (filter_buffer.cc:
       * 508-545); several parts into a growable buffer are not modelled
       * (TDBG_E_UNSUPPORTED, parity unpinned) */
      uint32_t ts = (uint32_t)oracle_datatype_size(f->datatype), bw = (uint32_t)f->byte_width;
      if ((ts != 4 && ts != 8) || (bw != 1 && bw != 2 && bw != 4 && bw != 8))
        return TDBG_E_UNSUPPORTED;
      uint32_t np;
      if ((rc = md_read(md, &np, 4))) return rc;
      uint64_t ip = 0, op = 0;
      for (uint32_t i = 0; i < np; i++) {
        uint32_t ps;
        if ((rc = md_read(md, &ps, 4))) return rc;
        if (ip + ps > in_n) return TDBG_E_DATA_READ;
        uint64_t ne = ps / bw;
        if (i > 0) return out->fixed ? TDBG_E_OUT_FULL : TDBG_E_UNSUPPORTED;
        if ((rc = out_prepend(out, ne * ts))) return rc;
        fscale_rev(ts, bw, f->scale, f->offset, in + ip, ne, out->p);
        op = ne * ts;
        ip += ps;
      }
      finish_size(out, op);
      return TDBG_OK;
    }
    case TDBG_FILTER_BYTESHUFFLE:
    case TDBG_FILTER_BITSHUFFLE:
    case TDBG_FILTER_XOR: {
      /* byteshuffle_filter.cc:111-147, bitshuffle_filter.cc:168-212,
       * xor_filter.cc:220-256 (same md / part walk) */
      uint32_t ts = (uint32_t)oracle_datatype_size(f->datatype);
      if (f->type == TDBG_FILTER_XOR && ts != 1 && ts != 2 && ts != 4 && ts != 8)
        return TDBG_E_UNSUPPORTED; /* "datatype size cannot be converted" */
      uint32_t np;
      if ((rc = md_read(md, &np, 4))) return rc;
      if ((rc = out_prepend(out, in_n))) return rc;
      uint64_t ip = 0;
      for (uint32_t i = 0; i < np; i++) {
        uint32_t ps;
        if ((rc = md_read(md, &ps, 4))) return rc;
        if (ip + ps > in_n) return TDBG_E_DATA_READ; /* get_const_buffer */
        if (f->type == TDBG_FILTER_BYTESHUFFLE)
          oracle_byteshuffle(1, ts, in + ip, ps, out->p + ip);
        else if (f->type == TDBG_FILTER_XOR)
          xor_part(1, ts, in + ip, ps, out->p + ip);
        else if (ps % ts != 0 || ps % 8 != 0)
          memcpy(out->p + ip, in + ip, ps);
        else
          bitshuffle_part(1, ts, in + ip, ps, out->p + ip);
        ip += ps;
      }
      finish_size(out, ip);
      return TDBG_OK;
    }
    case TDBG_FILTER_BIT_WIDTH_REDUCTION: {
      ival_t t = bwr_type(f->datatype, p->version);
      if (!t.active) PASS_THROUGH();
      /* bwr.cc:352-404 */
      uint32_t dts = (uint32_t)oracle_datatype_size(f->datatype);
      uint32_t orig, nw;
      if ((rc = md_read(md, &orig, 4))) return rc;
      if ((rc = md_read(md, &nw, 4))) return rc;
      if ((rc = out_prepend(out, orig))) return rc;
      uint64_t ip = 0, op = 0;
      for (uint32_t k = 0; k < nw; k++) {
        uint64_t off = 0;
        uint8_t bits;
        uint32_t nb;
        if ((rc = md_read(md, &off, dts))) return rc;
        if ((rc = md_read(md, &bits, 1))) return rc;
        if ((rc = md_read(md, &nb, 4))) return rc;
        if (bits >= 8 * t.w || nb % t.w != 0) {
          if ((rc = copy_in_out(in, in_n, ip, out, &op, nb))) return rc;
          ip += nb;
        } else {
          if (bits != 8 && bits != 16 && bits != 32 && bits != 64) return TDBG_E_BWR_BITS;
          uint32_t cb = bits / 8;
          for (uint32_t j = 0; j < nb / t.w; j++) {
            if (ip + cb > in_n) return TDBG_E_DATA_READ;
            uint64_t v = ld(in + ip, cb);
            ip += cb;
            if (t.sgn) v = (uint64_t)sext(v, cb);
            v = (v + off) & mask_w(t.w);
            if (op + dts > out->cap) return TDBG_E_OUT_FULL;
            st(out->p + op, v, dts);
            op += dts;
          }
        }
      }
      finish_size(out, op);
      return TDBG_OK;
    }
    case TDBG_FILTER_POSITIVE_DELTA: {
      ival_t t = pd_type(f->datatype, p->version);
      if (!t.active) PASS_THROUGH();
      /* pd.cc:324-375 */
      uint32_t dts = (uint32_t)oracle_datatype_size(f->datatype);
      uint32_t nw;
      if ((rc = md_read(md, &nw, 4))) return rc;
      if ((rc = out_prepend(out, in_n))) return rc;
      uint64_t ip = 0, op = 0;
      for (uint32_t k = 0; k < nw; k++) {
        uint64_t first = 0;
        uint32_t nb;
        if ((rc = md_read(md, &first, dts))) return rc;
        if ((rc = md_read(md, &nb, 4))) return rc;
        if (nb % t.w != 0) {
          if ((rc = copy_in_out(in, in_n, ip, out, &op, nb))) return rc;
          ip += nb;
        } else {
          uint64_t prev = first;
          for (uint32_t j = 0; j < nb / t.w; j++) {
            if (ip + t.w > in_n) return TDBG_E_DATA_READ;
            uint64_t d = ld(in + ip, t.w);
            ip += t.w;
            uint64_t v = (prev + d) & mask_w(t.w);
            if (op + dts > out->cap) return TDBG_E_OUT_FULL;
            st(out->p + op, v, dts);
            op += dts;
            prev = v;
          }
        }
      }
      finish_size(out, op);
      return TDBG_OK;
    }
    case TDBG_FILTER_RLE:
    case TDBG_FILTER_DELTA:
    case TDBG_FILTER_DOUBLE_DELTA: {
      if (f->compressor == TDBG_COMPRESSOR_NONE) PASS_THROUGH();
      /* compression_filter.cc:303-347, 413-486 */
      uint32_t nmd, nd;
      if ((rc = md_read(md, &nmd, 4))) return rc;
      if ((rc = md_read(md, &nd, 4))) return rc;
      if (!out->fixed) { out->p = NULL; out->cap = 0; out->size = 0; out->owned = 1; }
      uint8_t* mdb = NULL;
      uint64_t mdcap = 0, mdo = 0, op = 0, ip = 0;
      uint8_t ddt = f->reinterpret != TDBG_ANY ? f->reinterpret : f->datatype;
      for (uint32_t i = 0; i < nmd + nd; i++) {
        uint32_t un, cn;
        int is_md = i < nmd;
        if ((rc = md_read(md, &un, 4))) goto fail;
        if ((rc = md_read(md, &cn, 4))) goto fail;
        uint8_t* dst;
        if (is_md) {
          mdb = (uint8_t*)realloc(mdb, mdcap + un + 1);
          memset(mdb + mdcap, 0, un + 1);
          mdcap += un;
          dst = mdb + mdo;
        } else if (out->fixed) {
          if (op + un > out->cap) { rc = TDBG_E_OUT_FULL; goto fail; }
          dst = out->p + op;
        } else {
          out->p = (uint8_t*)realloc(out->p, out->cap + un + 1);
          memset(out->p + out->cap, 0, un + 1);
          out->cap += un;
          dst = out->p + op;
        }
        if (ip + cn > in_n) { rc = TDBG_E_DATA_READ; goto fail; }
        uint64_t wr;
        if (f->type == TDBG_FILTER_RLE)
          rc = rle_decompress_w(p->cell_size, in + ip, cn, dst, un, &wr);
        else if (f->type == TDBG_FILTER_DELTA)
          rc = delta_decompress_w(ddt, in + ip, cn, dst, un, &wr);
        else
          rc = dd_decompress_w(ddt, in + ip, cn, dst, un, &wr);
        if (rc) goto fail;
        if (is_md) mdo += un; else op += un;
        ip += cn;
      }
      *newmd = mdb;
      *newmd_n = mdo;
      *md_replaced = 1;
      if (out->fixed) out->size = out->cap;
      else out->size = op;
      return TDBG_OK;
    fail:
      free(mdb);
      return rc;
    }
    default:
      if (is_compression_type(f->type) && f->compressor == TDBG_COMPRESSOR_NONE)
        PASS_THROUGH();
      return TDBG_E_UNSUPPORTED;
  }
#undef PASS_THROUGH
}

/* FilterPipeline::run_reverse for one chunk (filter_pipeline.cc:449-514). */
static int rev_chunk(const oracle_pipeline* p, const uint8_t* md, uint64_t mdn,
                     const uint8_t* data, uint64_t dn, uint8_t* out,
                     uint64_t orig) {
  if (p->nfilters == 0) {
    /* input_data.copy_to(output) -- guarded here against overrun */
    if (dn > orig) return TDBG_E_OUT_FULL;
    memcpy(out, data, dn);
    return TDBG_OK;
  }
  const uint8_t* cin = data;
  uint64_t cin_n = dn;
  uint8_t* cin_owned = NULL;
  uint8_t* md_owned = NULL;
  mdcur_t c = {md, mdn, 0};
  int rc = TDBG_OK;
  for (int k = (int)p->nfilters - 1; k >= 0; k--) {
    obuf_t o = {0};
    if (k == 0) { o.p = out; o.cap = orig; o.size = orig; o.fixed = 1; }
    uint8_t* nm = NULL;
    uint64_t nmn = 0;
    int repl = 0;
    c.off = 0;
    rc = rev_filter(p, &p->f[k], cin, cin_n, &c, &o, &nm, &nmn, &repl);
    if (rc) {
      if (o.owned && o.p != cin) free(o.p);
      break;
    }
    if (repl) {
      free(md_owned);
      md_owned = nm;
      c.p = nm;
      c.n = nmn;
      c.off = 0;
    } else {
      /* output metadata = view of the unread remainder (e.g.
       * byteshuffle_filter.cc:143-145) */
      c.p += c.off;
      c.n -= c.off;
      c.off = 0;
    }
    if (k > 0) {
      if (o.owned) {
        free(cin_owned);
        cin_owned = o.p;
      }
      cin = o.p;
      cin_n = o.size;
    }
  }
  free(cin_owned);
  free(md_owned);
  return rc;
}

int oracle_unfilter_tile(const oracle_pipeline* p, const uint8_t* f,
                         uint64_t fsize, uint8_t* out, uint64_t out_size,
                         int is_offsets) {
  if (!p || (!f && fsize) || (!out && out_size)) return TDBG_E_ARG;
  uint64_t expected = out_size;
  if (is_offsets) {
    if (out_size < 8) return TDBG_E_TILE_SIZE; /* tile.cc:244-246 */
    expected = out_size - 8;
  }
  /* Tile::load_chunk_data tile.cc:280-313 */
  if (fsize < 8) return TDBG_E_TILE_FORMAT;
  uint64_t nch = ld(f, 8), o = 8, total = 0;
  /* first pass: directory */
  for (uint64_t i = 0; i < nch; i++) {
    if (o + 12 > fsize) return TDBG_E_TILE_FORMAT;
    uint64_t orig = ld(f + o, 4), fl = ld(f + o + 4, 4), ml = ld(f + o + 8, 4);
    o += 12;
    if (ml > fsize - o) return TDBG_E_TILE_FORMAT;
    o += ml;
    if (fl > fsize - o) return TDBG_E_TILE_FORMAT;
    o += fl;
    total += orig;
  }
  if (total != expected) return TDBG_E_TILE_SIZE;
  o = 8;
  uint64_t coff = 0;
  for (uint64_t i = 0; i < nch; i++) {
    uint64_t orig = ld(f + o, 4), fl = ld(f + o + 4, 4), ml = ld(f + o + 8, 4);
    o += 12;
    int rc = rev_chunk(p, f + o, ml, f + o + ml, fl, out + coff, orig);
    if (rc) return rc;
    o += ml + fl;
    coff += orig;
  }
  return TDBG_OK;
}

/* ------------------------------------------------------------------------ */
/* multi-threaded batch (CPU baseline)                                       */
/* ------------------------------------------------------------------------ */
typedef struct {
  const oracle_pipeline* p;
  uint64_t lo, hi;
  const uint8_t* in_base;
  const uint64_t *in_off, *in_size, *out_off, *out_size;
  uint8_t* out_base;
  int32_t* status;
} mt_job_t;

static void* mt_worker(void* arg) {
  mt_job_t* j = (mt_job_t*)arg;
  for (uint64_t i = j->lo; i < j->hi; i++)
    j->status[i] = oracle_unfilter_tile(j->p, j->in_base + j->in_off[i], j->in_size[i],
                                        j->out_base + j->out_off[i], j->out_size[i], 0);
  return NULL;
}

int oracle_unfilter_tiles_mt(const oracle_pipeline* p, uint64_t ntiles,
                             const uint8_t* in_base, const uint64_t* in_off,
                             const uint64_t* in_size, uint8_t* out_base,
                             const uint64_t* out_off, const uint64_t* out_size,
                             int nthreads, int32_t* status) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  mt_job_t jobs[256];
  /* parallel_for equal subranges (parallel_functions.h:171-284) */
  for (int t = 0; t < nthreads; t++) {
    jobs[t].p = p;
    jobs[t].lo = ntiles * (uint64_t)t / (uint64_t)nthreads;
    jobs[t].hi = ntiles * (uint64_t)(t + 1) / (uint64_t)nthreads;
    jobs[t].in_base = in_base;
    jobs[t].in_off = in_off;
    jobs[t].in_size = in_size;
    jobs[t].out_base = out_base;
    jobs[t].out_off = out_off;
    jobs[t].out_size = out_size;
    jobs[t].status = status;
    pthread_create(&th[t], NULL, mt_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  for (uint64_t i = 0; i < ntiles; i++)
    if (status[i]) return status[i];
  return TDBG_OK;
}
