/* ivc_oracle.c — plain-C restatement of the reference's motion estimation and motion
 * compensation.  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): used by tests/ as the
 * checker at frame sizes where the Python loop is too slow, and never linked into the
 * product.  Built by oracle/Makefile (gcc -O2 -ffp-contract=off).
 *
 * Follows /root/reference/ivclab/video/motion.py:
 *   compute_motion_vector  :8-58   (candidates dy outer / dx inner in [-sr, sr], skip
 *                                   out-of-frame windows :41-43, SSD = np.sum((block -
 *                                   ref_block) ** 2) :46 in the input dtype, first strict
 *                                   minimum :48, index (dy+sr)(2sr+1)+(dx+sr) :55)
 *   reconstruct_with_motion_vector :60-97 (block copy, zeros out of frame :89-92)
 * NumPy semantics of the SSD line: integer dtypes wrap in the subtraction and the square
 * and are summed exactly in a 64-bit accumulator (np.sum default dtype); float dtypes are
 * summed with NumPy's pairwise order for 64 contiguous elements: eight column
 * accumulators down the rows, then ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)).
 */
#include <stdint.h>
#include <string.h>
#include <math.h>

enum { U8 = 1, I8, U16, I16, U32, I32, U64, I64, F32, F64 };

/* SSD of one candidate, integer dtypes: wrap to the element width after sub and square */
#define DEF_INT_SSD(NAME, T, UT, ACC)                                                   \
  static ACC NAME(const T* cur, const T* ref, long W, long y, long x, long ry, long rx) { \
    ACC s = 0;                                                                          \
    for (int u = 0; u < 8; ++u)                                                         \
      for (int v = 0; v < 8; ++v) {                                                     \
        UT d = (UT)((UT)cur[(y + u) * W + x + v] - (UT)ref[(ry + u) * W + rx + v]);     \
        UT q = (UT)((uint64_t)d * (uint64_t)d); /* no int promotion: d*d overflows int */ \
        s = (ACC)((uint64_t)s + (uint64_t)(ACC)(T)q);                                   \
      }                                                                                 \
    return s;                                                                           \
  }
DEF_INT_SSD(ssd_u8, uint8_t, uint8_t, uint64_t)
DEF_INT_SSD(ssd_i8, int8_t, uint8_t, int64_t)
DEF_INT_SSD(ssd_u16, uint16_t, uint16_t, uint64_t)
DEF_INT_SSD(ssd_i16, int16_t, uint16_t, int64_t)
DEF_INT_SSD(ssd_u32, uint32_t, uint32_t, uint64_t)
DEF_INT_SSD(ssd_i32, int32_t, uint32_t, int64_t)
DEF_INT_SSD(ssd_u64, uint64_t, uint64_t, uint64_t)
DEF_INT_SSD(ssd_i64, int64_t, uint64_t, int64_t)

#define DEF_FLT_SSD(NAME, T)                                                            \
  static T NAME(const T* cur, const T* ref, long W, long y, long x, long ry, long rx) {  \
    T r[8];                                                                             \
    for (int v = 0; v < 8; ++v) {                                                       \
      T d = cur[y * W + x + v] - ref[ry * W + rx + v];                                  \
      r[v] = d * d;                                                                     \
    }                                                                                   \
    for (int u = 1; u < 8; ++u)                                                         \
      for (int v = 0; v < 8; ++v) {                                                     \
        T d = cur[(y + u) * W + x + v] - ref[(ry + u) * W + rx + v];                    \
        r[v] = r[v] + d * d;                                                            \
      }                                                                                 \
    return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));          \
  }
DEF_FLT_SSD(ssd_f32, float)
DEF_FLT_SSD(ssd_f64, double)

/* exact SSD of integer-valued uint8 frames (= the float64 computation, no wrap) */
static int64_t ssd_u8x(const uint8_t* cur, const uint8_t* ref, long W, long y, long x, long ry,
                       long rx) {
  int64_t s = 0;
  for (int u = 0; u < 8; ++u)
    for (int v = 0; v < 8; ++v) {
      int d = (int)cur[(y + u) * W + x + v] - (int)ref[(ry + u) * W + rx + v];
      s += d * d;
    }
  return s;
}

#define SEARCH_INT(FN, T, ACC)                                                          \
  {                                                                                     \
    const T* R = (const T*)ref; const T* Cc = (const T*)cur;                            \
    ACC best = 0; int have = 0;                                                         \
    for (int dy = -sr; dy <= sr; ++dy)                                                  \
      for (int dx = -sr; dx <= sr; ++dx) {                                              \
        long ry = y + dy, rx = x + dx;                                                  \
        if (ry < 0 || ry + 8 > H || rx < 0 || rx + 8 > W) continue;                     \
        ACC s = FN(Cc, R, W, y, x, ry, rx);                                             \
        if (!have || s < best) { best = s; have = 1; bdy = dy; bdx = dx; }              \
      }                                                                                 \
  }
#define SEARCH_FLT(FN, T)                                                               \
  {                                                                                     \
    const T* R = (const T*)ref; const T* Cc = (const T*)cur;                            \
    T best = (T)INFINITY;                                                               \
    for (int dy = -sr; dy <= sr; ++dy)                                                  \
      for (int dx = -sr; dx <= sr; ++dx) {                                              \
        long ry = y + dy, rx = x + dx;                                                  \
        if (ry < 0 || ry + 8 > H || rx < 0 || rx + 8 > W) continue;                     \
        T s = FN(Cc, R, W, y, x, ry, rx);                                               \
        if (s < best) { best = s; bdy = dy; bdx = dx; }                                 \
      }                                                                                 \
  }

/* mv for block rows [by0, by1) of one frame pair; mv has (by1-by0) x (W/8) entries.
 * mode 1 = exact SSD of u8 storage.  Returns 0, or -1 on a bad dtype. */
int oracle_me(const void* ref, const void* cur, int dtype, int mode, long H, long W, int sr,
              long by0, long by1, int64_t* mv) {
  long w = W / 8, n = 2 * sr + 1;
  for (long by = by0; by < by1; ++by)
    for (long bx = 0; bx < w; ++bx) {
      long y = 8 * by, x = 8 * bx;
      int bdy = 0, bdx = 0;
      if (mode == 1) {
        if (dtype != U8) return -1;
        SEARCH_INT(ssd_u8x, uint8_t, int64_t)
      } else {
        switch (dtype) {
          case U8: SEARCH_INT(ssd_u8, uint8_t, uint64_t) break;
          case I8: SEARCH_INT(ssd_i8, int8_t, int64_t) break;
          case U16: SEARCH_INT(ssd_u16, uint16_t, uint64_t) break;
          case I16: SEARCH_INT(ssd_i16, int16_t, int64_t) break;
          case U32: SEARCH_INT(ssd_u32, uint32_t, uint64_t) break;
          case I32: SEARCH_INT(ssd_i32, int32_t, int64_t) break;
          case U64: SEARCH_INT(ssd_u64, uint64_t, uint64_t) break;
          case I64: SEARCH_INT(ssd_i64, int64_t, int64_t) break;
          case F32: SEARCH_FLT(ssd_f32, float) break;
          case F64: SEARCH_FLT(ssd_f64, double) break;
          default: return -1;
        }
      }
      mv[(by - by0) * w + bx] = (bdy + sr) * n + (bdx + sr);
    }
  return 0;
}

/* motion.py:60-97 for one frame [H][W][C] of elem_size-byte elements */
void oracle_mc(const void* ref, int elem_size, long H, long W, long C, const int64_t* mv, int sr,
               void* out) {
  long n = 2 * sr + 1, row = W * C * elem_size;
  const uint8_t* R = (const uint8_t*)ref;
  uint8_t* O = (uint8_t*)out;
  memset(O, 0, (size_t)(H * row));
  for (long by = 0; by < H / 8; ++by)
    for (long bx = 0; bx < W / 8; ++bx) {
      int64_t idx = mv[by * (W / 8) + bx];
      /* Python floor division / modulo */
      int64_t q = idx / n, r = idx % n;
      if (r < 0) { r += n; q -= 1; }
      long dy = (long)q - sr, dx = (long)r - sr;
      long ry = 8 * by + dy, rx = 8 * bx + dx;
      if (ry < 0 || ry + 8 > H || rx < 0 || rx + 8 > W) continue;
      for (int u = 0; u < 8; ++u)
        memcpy(O + (8 * by + u) * row + 8 * bx * C * elem_size,
               R + (ry + u) * row + rx * C * elem_size, (size_t)(8 * C * elem_size));
    }
}
