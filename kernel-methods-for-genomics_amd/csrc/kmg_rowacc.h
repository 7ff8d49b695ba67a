// kmg_rowacc.h — shared pieces of the row-accumulator Gram kernels (kmg_gram.hip,
// kmg_nbhd.hip): a workgroup accumulates one row of K (one column chunk) in LDS, then
// streams it to HBM.  Device code only; included by the .hip translation units.
#pragma once
#include "kmg_internal.h"

namespace kmg {

// Workgroup -> (column chunk c, local row il) of the row-accumulator grids, chunk-major.
// With o.tri (a full square K) chunk c keeps only the rows i < col0(c) + cw(c), the blocks
// that reach the diagonal or lie right of it: K is symmetric, and the blocks left of row
// i's own chunk are mirrored afterwards (launch_mirror_chunks), so a row reads the posting
// lines of (nch + 1) / 2 chunks on average instead of nch.  rowacc_blocks() is the grid size.
__host__ __device__ __forceinline__ int64_t tri_rows(int64_t n, int chunk, int c, int64_t row0,
                                                    int64_t rows) {
  const int64_t end = min(n, (int64_t)(c + 1) * chunk) - row0;
  return end < 0 ? 0 : (end < rows ? end : rows);
}
__host__ __device__ __forceinline__ int64_t rowacc_blocks(const IndexGeom &g, const OutSpec &o,
                                                         int64_t row0, int64_t rows) {
  if (!o.tri) return rows * g.nchunks;
  int64_t t = 0;
  for (int c = 0; c < g.nchunks; ++c) t += tri_rows(g.n, g.chunk, c, row0, rows);
  return t;
}
__device__ __forceinline__ void rowacc_item(const IndexGeom &g, const OutSpec &o, int64_t row0,
                                            int64_t rows, int64_t b, int &c, int64_t &il) {
  if (!o.tri) {
    c = (int)(b / rows);
    il = b - (int64_t)c * rows;
    return;
  }
  for (c = 0; c < g.nchunks - 1; ++c) {
    const int64_t rc = tri_rows(g.n, g.chunk, c, row0, rows);
    if (b < rc) break;
    b -= rc;
  }
  il = b;
}
// (item b = blockIdx.x: one workgroup per item)
__device__ __forceinline__ void rowacc_block(const IndexGeom &g, const OutSpec &o, int64_t row0,
                                             int64_t rows, int &c, int64_t &il) {
  rowacc_item(g, o, row0, rows, (int64_t)blockIdx.x, c, il);
}

// copy the packed record of sequence i into LDS (every thread of the block takes part)
__device__ __forceinline__ void stage_record(const Packed &pk, int64_t i, uint32_t *srec) {
  const uint32_t *rec = pk.w + i * pk.ldp;
  for (int t = threadIdx.x; t < (int)pk.ldp; t += blockDim.x) srec[t] = rec[t];
}

// ------------------------------------------------------------------ epilogue
template <int DT, bool NT = false>
__device__ __forceinline__ void emit4(const OutSpec &o, int64_t il, int64_t ig, int64_t col,
                                      int cnt, int64_t v0, int64_t v1, int64_t v2, int64_t v3,
                                      bool norm) {
  const int64_t v[4] = {v0, v1, v2, v3};
  if constexpr (DT == KMG_I32) {
    int32_t *p = (int32_t *)o.out + il * o.ld + col;
    if (cnt == 4 && ((uintptr_t)p & 15) == 0) {
      typedef int v4i __attribute__((ext_vector_type(4)));
      const v4i x = {(int)v0, (int)v1, (int)v2, (int)v3};
      if constexpr (NT)
        __builtin_nontemporal_store(x, (v4i *)p);
      else
        *(v4i *)p = x;
    } else {
      for (int q = 0; q < cnt; ++q) p[q] = (int32_t)v[q];
    }
  } else {
    double r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < cnt) {
        if (norm) {
          // normalize_K: K[i,j] /= (d * diag[j]) with d = sqrt(K[i,i]); diagonal := 1
          const int64_t cs = o.col_seq0 + col + q;
          r[q] = (ig == cs) ? 1.0 : (double)v[q] / (o.dsq[ig] * o.dsq[cs]);
        } else {
          r[q] = (double)v[q];
        }
      } else {
        r[q] = 0.0;
      }
    }
    if constexpr (DT == KMG_F64) {
      double *p = (double *)o.out + il * o.ld + col;
      if (cnt == 4 && ((uintptr_t)p & 15) == 0) {
        if constexpr (NT) {
          typedef double v2d __attribute__((ext_vector_type(2)));
          const v2d a = {r[0], r[1]}, b = {r[2], r[3]};
          __builtin_nontemporal_store(a, (v2d *)p);
          __builtin_nontemporal_store(b, (v2d *)(p + 2));
        } else {
          *(double2 *)p = make_double2(r[0], r[1]);
          *(double2 *)(p + 2) = make_double2(r[2], r[3]);
        }
      } else {
        for (int q = 0; q < cnt; ++q) p[q] = r[q];
      }
    } else {
      float *p = (float *)o.out + il * o.ld + col;
      if (cnt == 4 && ((uintptr_t)p & 15) == 0) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        const v4f x = {(float)r[0], (float)r[1], (float)r[2], (float)r[3]};
        if constexpr (NT)
          __builtin_nontemporal_store(x, (v4f *)p);
        else
          *(v4f *)p = x;
      } else {
        for (int q = 0; q < cnt; ++q) p[q] = (float)r[q];
      }
    }
  }
}

// Stream one int32 LDS accumulator row [0, cw) to K row il (columns col0 ..): 16 bytes per
// lane and step, so every store instruction of a wave covers 1 KB of the row contiguously
// (int32 / float32: 4 columns a lane, float64: 2).  Two 16-byte stores 32 bytes apart per
// lane (emit4's float64 form) leave half-written lines behind every store instruction,
// which cost the spectrum kernel 2.2x as non-temporal stores (profiles/r02t_sp_store.jsonl).
// A16: the counters are packed 16-bit (column q at halfword q of the accumulator)
template <bool NT, bool A16 = false>
__device__ __forceinline__ void emit_row(const OutSpec &o, int64_t il, int64_t i, int64_t col0,
                                         int cw, const int32_t *acc, bool norm) {
  const uint16_t *a16 = (const uint16_t *)acc;
  // columns below o.col_lo are not written; col_lo - col0 is a multiple of 8 (host check)
  const int qs = (int)max((int64_t)0, o.col_lo - col0);
  if (o.dtype == KMG_U8) {
    // raw off-diagonal counts as uint8 (the diagonal column is stored as 0: the unpack takes
    // K_ii from the diagonal), 16 columns = 16 B per lane and step; an off-diagonal count
    // >= 255 goes to the escape list (or, with none / a full one, is flagged and the caller
    // redoes the build with 16-bit slabs)
    uint8_t *prow = (uint8_t *)o.out + il * o.ld + col0;
    bool big = false;
    for (int q = qs + threadIdx.x * 16; q < cw; q += blockDim.x * 16) {
      uint32_t v[16];
#pragma unroll
      for (int h = 0; h < 16; ++h) {
        const uint32_t x = q + h < cw ? (A16 ? (uint32_t)a16[q + h] : (uint32_t)acc[q + h]) : 0u;
        const bool dg = o.col_seq0 + col0 + q + h == i;
        v[h] = (dg || q + h >= cw) ? 0u : u8_slab_entry(o, i, col0 + q + h, x, big);
      }
      uint8_t *d = prow + q;
      if (q + 16 <= cw && (((uintptr_t)d) & 15) == 0) {
        uint4 x;
        x.x = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
        x.y = v[4] | (v[5] << 8) | (v[6] << 16) | (v[7] << 24);
        x.z = v[8] | (v[9] << 8) | (v[10] << 16) | (v[11] << 24);
        x.w = v[12] | (v[13] << 8) | (v[14] << 16) | (v[15] << 24);
        *(uint4 *)d = x;
      } else {
        for (int h = 0; h < 16 && q + h < cw; ++h) d[h] = (uint8_t)v[h];
      }
    }
    if (big && o.ovf) atomicOr(o.ovf, 1u);
    return;
  }
  if (o.dtype == KMG_U16) {
    // raw counts as uint16 (multi-GPU round slabs; no normalisation here: the unpack pass
    // applies it), 8 columns = 16 B per lane and step; a count above 65535 is clipped and
    // flagged, and the caller redoes the build with 32-bit slabs
    uint16_t *prow = (uint16_t *)o.out + il * o.ld + col0;
    bool big = false;
    for (int q = qs + threadIdx.x * 8; q < cw; q += blockDim.x * 8) {
      uint32_t v[8];
      if (q + 8 <= cw) {
        if constexpr (A16) {
          const uint4 a = *(const uint4 *)&a16[q];
          v[0] = a.x & 0xFFFFu; v[1] = a.x >> 16; v[2] = a.y & 0xFFFFu; v[3] = a.y >> 16;
          v[4] = a.z & 0xFFFFu; v[5] = a.z >> 16; v[6] = a.w & 0xFFFFu; v[7] = a.w >> 16;
        } else {
          const uint4 a = *(const uint4 *)&acc[q], b = *(const uint4 *)&acc[q + 4];
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
          v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        }
      } else {
#pragma unroll
        for (int h = 0; h < 8; ++h) v[h] = q + h < cw ? (A16 ? (uint32_t)a16[q + h] : (uint32_t)acc[q + h]) : 0u;
      }
#pragma unroll
      for (int h = 0; h < 8; ++h) {
        big |= v[h] > 0xFFFFu;
        v[h] = min(v[h], 0xFFFFu);
      }
      uint16_t *d = prow + q;
      if (q + 8 <= cw && (((uintptr_t)d) & 15) == 0) {
        const uint4 x = make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16),
                                   v[6] | (v[7] << 16));
        if constexpr (NT) {
          typedef int v4i __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(__builtin_bit_cast(v4i, x), (v4i *)d);
        } else {
          *(uint4 *)d = x;
        }
      } else {
        for (int h = 0; h < 8 && q + h < cw; ++h) d[h] = (uint16_t)v[h];
      }
    }
    if (big && o.ovf) atomicOr(o.ovf, 1u);
    return;
  }
  if (o.dtype == KMG_F64) {
    typedef double v2d __attribute__((ext_vector_type(2)));
    double *prow = (double *)o.out + il * o.ld + col0;
    const bool al = (((uintptr_t)prow) & 15) == 0;
    const double di = norm ? o.dsq[i] : 1.0;
    for (int q = qs + threadIdx.x * 2; q < cw; q += blockDim.x * 2) {
      int2 w;
      if constexpr (A16) {
        const uint32_t pr = *(const uint32_t *)&a16[q];
        w = make_int2((int)(pr & 0xFFFFu), (int)(pr >> 16));
      } else {
        w = *(const int2 *)&acc[q];
      }
      const int64_t c0 = o.col_seq0 + col0 + q;  // the column's sequence
      const bool two = q + 1 < cw;
      double r0 = (double)w.x, r1 = two ? (double)w.y : 0.0;
      if (norm) {  // normalize_K: K[i,j] / (sqrt(K[i,i]) * sqrt(K[j,j])), diagonal := 1
        r0 = (i == c0) ? 1.0 : (double)w.x / (di * o.dsq[c0]);
        r1 = !two ? 0.0 : (i == c0 + 1) ? 1.0 : (double)w.y / (di * o.dsq[c0 + 1]);
      }
      if (al && two) {
        const v2d x = {r0, r1};
        if constexpr (NT)
          __builtin_nontemporal_store(x, (v2d *)(prow + q));
        else
          *(v2d *)(prow + q) = x;
      } else {
        prow[q] = r0;
        if (two) prow[q + 1] = r1;
      }
    }
  } else {
    for (int q = qs + threadIdx.x * 4; q < cw; q += blockDim.x * 4) {
      int4 w;
      if constexpr (A16) {
        const uint2 pr = *(const uint2 *)&a16[q];
        w = make_int4((int)(pr.x & 0xFFFFu), (int)(pr.x >> 16), (int)(pr.y & 0xFFFFu), (int)(pr.y >> 16));
      } else {
        w = *(const int4 *)&acc[q];
      }
      if (o.dtype == KMG_F32)
        emit4<KMG_F32, NT>(o, il, i, col0 + q, min(4, cw - q), w.x, w.y, w.z, w.w, norm);
      else
        emit4<KMG_I32, NT>(o, il, i, col0 + q, min(4, cw - q), w.x, w.y, w.z, w.w, norm);
    }
  }
}

// ------------------------------------------------------------------ mismatch m=1
// LDS byte address of the 16-bit column in halfword H of w (acc at LDS offset 0): one
// SDWA shift instead of extract + shift-add.
template <int H>
__device__ __forceinline__ uint32_t col_addr_sdwa(uint32_t w) {
  uint32_t r;
  if constexpr (H == 0)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
        "src1_sel:WORD_0"
        : "=v"(r)
        : "v"(w));
  else
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
        "src1_sel:WORD_1"
        : "=v"(r)
        : "v"(w));
  return r;
}

}  // namespace kmg
