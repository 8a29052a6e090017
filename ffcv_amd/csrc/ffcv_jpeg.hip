// ffcv_jpeg.hip -- baseline JPEG decode on gfx950, fused with the RRC crop,
// INTER_AREA resize and the flip / cutout / normalize epilogue.
//
// Reference: rgb_image.py:194-208 decodes every JPEG in full with
// libjpeg-turbo (libffcv.cpp:104-106: tjDecompress2(TJPF_RGB,
// TJFLAG_FASTDCT) = ifast IDCT + fancy upsampling + fixed-point YCbCr->RGB)
// into a temp buffer, then crops and resizes on the CPU.
//
// Launches per batch (launch_rrc): k1_order_kernel (size-sorted image order),
// then three kernels on the launch's stream:
//
// K1 jpeg_entropy_kernel -- ONE WAVE (64 lanes) per image, four images per
// 256-thread workgroup sharing one LDS table set (38.8 KB: 16 images per CU).
// (A self-synchronising Huffman decode costs about the same latency at 64 or
// 256 lanes per image -- the latency is the resynchronisation distance -- but
// a third of the lane-steps at 64, so the wave-per-image shape triples
// throughput.)
//   P0  gather (table[ids[k]]) and the RRC / cutout / flip draws (wave 0 for
//       the workgroup); the first 2 KB of the file staged in LDS; the whole
//       wave walks the markers (SOF/DHT/DQT/DRI/SOS) on wave-uniform values,
//       validates geometry and tables, and hands out Huffman table slots
//   P1  Huffman decode tables (jdhuff.c jpeg_make_d_derived_tbl, with its
//       checks): per slot an 11-bit (luma AC), 10-bit (chroma AC) or 8-bit
//       (DC) first-level LUT with two-symbol pair entries, a 5-bit second
//       level for longer codes, canonical limits for the rest; ifast
//       dequantisation multipliers (jddctmgr.c); built once per workgroup when
//       its images' tables agree, else per image in global scratch
//   P2  de-stuffing (0xFF00 -> 0xFF) of the entropy-coded segment in stream
//       order, one coalesced dword per lane per step with a wave scan of the
//       kept-byte counts, into an L2-resident scratch stream (zero-padded:
//       libjpeg fills zeros after a marker)
//   P3  self-synchronising parallel Huffman decode.  The stream is cut into
//       one bit range per lane; a lane decodes its range from a guessed state
//       (bit position, coefficient index z, block-in-MCU), records where its
//       blocks start, and the state at which it leaves the range.  Each
//       further round gives lane t the exit state of lane t-1; a lane whose
//       guess changed re-decodes only until it reaches a block start it
//       recorded before (same bit position and MCU phase: from there its old
//       trajectory is exact).  Lane 0 is exact, so round r fixes lanes 0..r
//       at worst; rounds end when no guess changes.  (The entropy index skips
//       these rounds for a sample decoded before.)
//   P4  wave scan of blocks-started -> each lane's first block index
//   P5  write pass: DC differences summed per lane, quantised AC coefficients
//       (zigzag order) of the blocks the crop window needs, into a zeroed
//       window; K2's resize plan and linear tap table
//
// K1b jpeg_idct_kernel -- one workgroup per image: DC prediction from the
//   per-lane sums, de-zigzag + dequantise + ifast IDCT (jidctfst.c) of the
//   window's blocks -> component planes in scratch.
//
// K2 jpeg_color_resize_kernel -- one workgroup per band of 16 output rows:
//   stages the band's plane tiles and then its source rows of the crop as RGB
//   in LDS (jdsample.c fancy upsampling + jdcolor.c fixed-point YCbCr->RGB,
//   once per source pixel), then computes the band's output pixels with the
//   OpenCV 4.5.4 resize restatement (linear walk, area walk, or the general
//   per-pixel path) + flip / cutout / LUT epilogue.
//
// Every integer step matches libjpeg-turbo bit for bit
// (tests/test_kernels_gpu.py); float steps use -ffp-contract=off.
#include <climits>

#include "api_internal.h"
#include "device_common.h"
#include "diag_hooks.h"

#define JT 64           // lanes per wave
// JL = 32 (two images per wave, each with twice the bits per lane) was
// bit-exact in round 1 but 12-35% slower than 64 (the longer per-image latency
// outweighed the ~25% fewer sync lane-steps); it is no longer maintained: a
// round-5 build (-DJL=32, 46 KB of LDS, 3 workgroups per CU) ran the C3 bench
// 10% slower and no longer matched the oracle (profiles/r5b_ab20_jl32.log).
#ifndef JL
#define JL 64           // lanes per image: a wave decodes JT / JL images side by side
#endif
static_assert(JL == JT, "JL != 64 is not maintained: a round-5 -DJL=32 build was 10% slower and not bit-exact (profiles/r5b_ab20_jl32.log)");
#define IPW (JT / JL)   // images per wave
#define HDR_BYTES 2048  // header bytes staged in LDS (aliased by the LUT pool)
#ifndef FB_AC
#define FB_AC 11        // first-level bits, the scan's first AC table (luma)
#endif
static_assert(FB_AC <= 11, "FB_AC > 11 is not supported: a 12-bit build failed the bench parity check (DESIGN.md s6, r6j)");
#define FB_AC2 10       // first-level bits, further AC tables (chroma)
#ifndef FB_DC
#define FB_DC 8         // first-level bits, DC tables
#endif
// first-level LUT words shared by the slots (+ two zero words): one table of
// each AC size and two DC tables, the 4:2:0 / 4:2:2 / 4:4:4 norm
#define LUT_POOL ((1 << FB_AC) + (1 << FB_AC2) + 2 * (1 << FB_DC) + 2)
#define SUBB 5          // second-level bits
#ifndef NSUB
#define NSUB 8          // second-level tables per slot
#endif
#define NSLOT 6         // Huffman tables a scan can reference (3 DC + 3 AC)
#define NLUTSLOT 4      // slots that can get a first-level LUT from the pool
#define NTAB 8
#ifndef NEV
#define NEV 6
#endif
#define DS_FLUSH 8      // de-stuff steps per LDS -> HBM flush
#define DS_DEPTH 8      // de-stuff loads in flight per lane
#define STAGE_BYTES (DS_FLUSH * JL * 4 + 64)  // a flush's bytes + the carried tail + pad
#define STAGE_DUMMY (STAGE_BYTES - 4)
#define STREAM_PAD 32   // zero bytes after the de-stuffed stream
#ifndef ACS_Z
#define ACS_Z 24        // zigzag positions of a block the write pass stages in LDS
#endif
#define ACS_BYTES (ACS_Z * 2)
#ifndef K1_CF_CPOL
// cache policy of K1's window-coefficient stores (zeroing, direct, flush):
// 0 default; A/B builds: 2 = nt, 16 = sc1 (write-through, the line leaves
// the XCD's L2: MI355X_MICROARCH.md, "stores of each flavour")
#define K1_CF_CPOL 0
#endif
#ifndef BAND
#define BAND 16  // K2 output rows per workgroup
#endif
#ifndef K2T
#define K2T 256  // K2 threads per workgroup
#endif
#define K2_COLS 128  // K2 fast path: output column-pair slots (out_w <= 256); K2T / K2_COLS row groups
#ifndef K2_LDS
#define K2_LDS 26624  // K2 dynamic LDS: the most that keeps 6 workgroups per CU (6 x 26 KB of 160 KB; 512 B granules); bigger bands take the general path (24 KB: 1% slower at C3, 32 KB: 3% slower)
#endif
#ifndef JW
#define JW 4  // waves per K1 workgroup
#endif
#ifndef K1_PAD
#define K1_PAD 0  // extra (unused) dynamic LDS per K1 workgroup: caps K1 workgroups per CU (A/B knob)
#endif

enum JMode { JM_RRC = 0, JM_FULL = 1, JM_COEF = 2 };

// Per-image geometry written by K1 for K2.
struct ImgInfo {
  int32_t status;
  int32_t W, H, ncomp, color_rgb;
  int32_t he[3], ve[3];  // expansion factors hmax/h, vmax/v
  int32_t cw[3], ch[3], stride[3];
  int32_t ri, rj, rh, rw;
  // arena offset of each component's window plane, minus (wy0 * 8 * stride +
  // wx0 * 8): plane sample (row, col) in absolute coordinates is at
  // arena + poff + row * stride + col (stride = window width in samples)
  uint64_t poff[3];
  uint64_t rgb_off;  // K2 band staging (crop rows as RGB) for bands wider than LDS
  // RRC: the crop's resize plan, and whether K1 wrote the image's linear tap
  // table (JpegArgs::taps: out_w column taps, flip applied, then out_h row
  // taps), computed once per image instead of once per K2 workgroup
  ResizePlan plan;
  int32_t taps;
  // K1 -> jpeg_idct_kernel: what the DC prediction and the IDCT need
  uint64_t cf_off;   // arena offset of the window coefficients
  uint64_t coff[3];  // first window block of each component in the coefficient region
  int32_t nblocks, bpm, mcux;
  int32_t hs[3], vs[3], wx0[3], wx1[3], wy0[3], wy1[3], qmax[3];
  int32_t blk_comp[10], blk_dx[10], blk_dy[10];
  // DC prediction (RRC / FULL): slot 0 of a window block holds the running sum,
  // per component, of the DC differences its decoding lane had read up to and
  // including it; the absolute DC adds that lane's offset (the sums of the
  // lanes before it).  lane_blk0[l]: first block lane l started (non-decreasing)
  uint32_t lane_blk0[64];
  int32_t lane_off[3][64];
  int16_t qmul[3][64] __attribute__((aligned(16)));
  // this image's launch-arena reservation [arena_base, arena_base +
  // arena_need) (need 0: none); read only by ffcv_jpeg_arena_regions
  uint64_t arena_base, arena_need;
};

#define K2_TAPS 512  // tap table entries per image: out_w + out_h <= 512 (tap_pack format)

// Huffman decode tables built from one image's DHT segments.  K1 runs JW
// images per workgroup; images whose tables (and table slots) are byte-
// identical to the workgroup's first valid image share ONE LDS copy -- the
// usual case, every encoder of a dataset writes the same tables -- and any
// other image builds its own copy in global scratch (L1/L2-resident).
struct JTables {
  uint32_t lim[NSLOT][17];  // left-justified end of length-l codes
  int32_t valoff[NSLOT][17];
  uint8_t vals[NSLOT][256];
  int nsub[NSLOT];
  int nvals[NSLOT];
  int bad;
  uint16_t sub_prefix[NSLOT][NSUB];
  // second-level tables (codes longer than the first level; make_entry format)
  uint16_t lut2[NLUTSLOT][NSUB][1 << SUBB];
  uint32_t lut[LUT_POOL];  // first-level LUT pool (single or pair entries, see make_pair)
};

// Per-image (per-wave) state.
struct JShared {
  int status;
  const uint8_t *src;  // the image's bytes (read by the workgroup's table build)
  int W, H, ncomp, hmax, vmax;
  int hs[3], vs[3], tq[3], td[3], ta[3], cid[3];
  int color_rgb;
  int mcux, mcuy, bpm, nblocks;
  int cw[3], ch[3], bw[3], bh[3];
  int blk_comp[10], blk_dx[10], blk_dy[10];
  // Huffman table slots referenced by the scan (AC first); per block-in-MCU
  // slot numbers packed 3 bits per phase; per slot LUT base and bits
  int nslots;
  int slot_tab[NSLOT];  // class * 4 + id
  uint32_t sinfo[NSLOT];  // see SI_* below
  uint32_t dcpack, acpack, acmask;
  uint32_t scan_off;
  uint32_t dqt_off[4];
  int dqt_prec[4], dqt_ok[4];
  uint32_t dht_off[NTAB];
  int dht_ok[NTAB];
  int saw_jfif, saw_adobe, adobe_transform;
  int restart;
  int ri, rj, rh, rw;
  int wx0[3], wx1[3], wy0[3], wy1[3];
  uint64_t coff[3];  // first window block of each component in the coefficient region
  uint64_t poff[3];  // see ImgInfo::poff
  uint32_t nwin;     // window blocks (all components)
  // this image's regions of the launch arena (bump-allocated after the parse)
  uint64_t ds_off, cf_off, dc_off, rgb_off;
  uint32_t ds_bytes, cf_bytes, dc_bytes;
  uint32_t dlen;
  int any;
  // per block-in-MCU (phase) record, read by the decode loops for the phase
  // that follows the current one: its DC / AC table sinfo, its own successor
  // (so the loops carry the next phase index instead of computing ph + 1 mod
  // bpm and its address every step), and the write pass's descriptor: block
  // index of MCU (0,0) in the component's window, blocks per MCU row step,
  // hs, and the window as MCU ranges [mx_lo, mx_hi] x [my_lo, my_hi]
  // (64 bytes: the record address is one shift-add from the phase index)
  struct __attribute__((aligned(16))) PhaseRec {
    uint32_t dinf, ainf;
    int next, pad;
    int4 pd0, pd1, pad2;
  } phr[10];
  int qmax[3];  // max |qmul| of the AC multipliers per component (the IDCT's 32-bit-product test)
  union __attribute__((aligned(16))) {
    uint8_t hdr[HDR_BYTES];       // P0-P1: the first header bytes
    uint32_t ev[2][NEV + 1][JL];  // P3: block-start events (pos << 4 | phase), double-buffered
    uint8_t stage[STAGE_BYTES];   // P2: de-stuffed bytes awaiting a flush
    uint4 acs[JL][ACS_BYTES / 16];  // P5: each lane's block of low-frequency AC coefficients
  };
};

struct K1Shared {
  JTables tab;
  JShared w[JW * IPW];
};

// zigzag index of each natural (row-major) coefficient position; the entropy
// pass stores coefficients in zigzag order
constexpr uint8_t kZigzagOfNatural[64] = {
    0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42, 3,  8,  12, 17, 25, 30,
    41, 43, 9,  11, 18, 24, 31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38,
    46, 51, 55, 60, 21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

__constant__ uint8_t c_natural[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

__constant__ int32_t c_aanscales[64] = {
    16384, 22725, 21407, 19266, 16384, 12873, 8867,  4520,  22725, 31521, 29692, 26722, 22725,
    17855, 12299, 6270,  21407, 29692, 27969, 25172, 21407, 16819, 11585, 5906,  19266, 26722,
    25172, 22654, 19266, 15137, 10426, 5315,  16384, 22725, 21407, 19266, 16384, 12873, 8867,
    4520,  12873, 17855, 16819, 15137, 12873, 10114, 6967,  3552,  8867,  12299, 11585, 10426,
    8867,  6967,  4799,  2446,  4520,  6270,  5906,  5315,  4520,  3552,  2446,  1247};

// ------------------------------------------------------------ bit reader --
// The de-stuffed stream: big-endian bytes read as 32-bit words from the
// image's scratch slot (L2-resident: written in P2, re-read every round),
// zero-padded by STREAM_PAD bytes so no read needs a bounds check.  The
// reader holds 33..64 valid bits plus the next word, loaded right after a
// refill and consumed at the following one (~5 symbols later), so a symbol
// (code <= 16 bits + <= 15 extra bits) never waits on memory.
// p as a wave-uniform (scalar-register) pointer: every lane of the wave
// holds the same value when one image maps to one wave.
template <class P>
FFCV_DEV P *wave_uniform(P *p) {
  if constexpr (JL != JT) return p;
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (P *)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

typedef const __attribute__((address_space(1))) uint8_t gbytes_t;  // global memory
// Non-temporal loads of file bytes through the global address space: a
// generic pointer compiles to flat loads, which count in both vmcnt and
// lgkmcnt and defeat the compiler's per-load waits (every prefetch waited).
FFCV_DEV uint8_t gld_u8(const uint8_t *p) { return __builtin_nontemporal_load((gbytes_t *)p); }
FFCV_DEV uint32_t gld_u32(const uint32_t *p) {
  return __builtin_nontemporal_load((const __attribute__((address_space(1))) uint32_t *)p);
}
struct BitReader {
  gbytes_t *w;
  uint64_t acc;
  int nb;
  uint32_t wo;   // byte offset of the word in nxt (32-bit: scalar base + vector offset loads)
  uint32_t nxt;  // raw (little-endian) next word: swapped only when used, so
                 // its load is waited for at the next refill, not here
  FFCV_DEV uint32_t word(uint32_t off) const { return *(const __attribute__((address_space(1))) uint32_t *)(w + off); }
  FFCV_DEV void init(const uint32_t *words, uint32_t p) {
    w = (gbytes_t *)words;
    wo = (p >> 5) * 4;
    uint32_t w0 = __builtin_bswap32(word(wo)), w1 = __builtin_bswap32(word(wo + 4));
    wo += 8;
    nxt = word(wo);
    acc = (((uint64_t)w0 << 32) | (uint64_t)w1) << (p & 31);
    nb = 64 - (int)(p & 31);
  }
  FFCV_DEV void consume(int n) {
    acc <<= n;
    nb -= n;
    if (nb <= 32) {
      acc |= (uint64_t)__builtin_bswap32(nxt) << (32 - nb);
      nb += 32;
      wo += 4;
      nxt = word(wo);
    }
  }
};



struct DecState {
  uint32_t pos;
  int z;   // 0: next symbol is a DC; else index of the next AC coefficient
  int ph;  // block index inside the MCU
};

// Symbol -> decode entry: bits consumed (code + extra bits, 1..31) | extra
// bits << 5 | coefficient advance << 9.  DC: size = symbol, z 0 -> 1.  AC:
// size = low nibble; z advances by run+1, by 16 for ZRL, past the block for
// EOB.  A LUT word with bits-consumed 0 is not an entry: 0 sends the decode
// to the canonical fallback, (n + 1) << 5 to second-level table n.
FFCV_DEV uint32_t make_entry(bool ac, int len, int sym) {
  int size, zinc;
  if (!ac) {
    size = sym;
    zinc = 1;
  } else {
    size = sym & 15;
    int r = sym >> 4;
    zinc = size ? r + 1 : (r == 15 ? 16 : 127);
  }
  return (uint32_t)(len + size) | ((uint32_t)size << 5) | ((uint32_t)zinc << 9);
}

// Canonical decode of a 16-bit lookahead (jdhuff.c jpeg_huff_decode): the
// code length is the first l with look < lim[l]; past lim[16] the code is
// invalid and, like libjpeg, yields symbol 0 after 16 bits.
template <class TB>
FFCV_DEV uint32_t slow_entry(const TB &T, uint32_t acmask, int slot, uint32_t look) {
  int len = 1;
#pragma unroll
  for (int l = 1; l < 16; l++) len += look >= T.lim[slot][l];
  int sym = 0;
  if (look < T.lim[slot][16]) sym = T.vals[slot][(T.valoff[slot][len] + (int)(look >> (16 - len))) & 0xff];
  else len = 16;
  return make_entry((acmask >> slot) & 1, len, sym);
}

// Two AC symbols per first-level lookup.  When a first-level AC entry's
// symbol (code + extra bits, t1 bits) is not EOB and the next symbol's code
// and extra bits also fit in the first-level window, the entry carries both:
//   [0:5) total bits  [5:9) size1  [9:16) z advance of both (clamped 127)
//   [16:21) t1  [21:25) size2  [25:32) z advance of the first (1..16)
// A single entry has bits 16.. zero.  A pair never crosses a block end:
// the decoder takes only the first symbol when it alone reaches z = 64.
// Then e >> 16 is the first symbol's entry for the sync pass (bits t1 in
// [0:5), advance in [9:16)), so both passes select with one shift.  The
// symbol sequence and every bit position are the same as decoding one
// symbol per step.
template <class TB>
FFCV_DEV uint32_t make_pair(const TB &T, int slot, int bits, const uint32_t *L, uint32_t look, uint32_t e1) {
  // L[l] = T.lim[slot][l] for l <= FB_AC, in registers
  const int t1 = (int)(e1 & 31), size1 = (int)(e1 >> 5) & 15, zinc1 = (int)(e1 >> 9);
  if (zinc1 > 16 || t1 >= bits) return e1;  // EOB, or no room for a second code
  const uint32_t look2 = (look << t1) & 0xffffu;
  const int room = bits - t1;
  int len = 1;  // the canonical length if it is at most room (limits are non-decreasing)
#pragma unroll
  for (int l = 1; l < FB_AC; l++) len += (l < room && look2 >= L[l]) ? 1 : 0;
  if (look2 >= T.lim[slot][len]) return e1;  // a longer code
  const int sym = T.vals[slot][(T.valoff[slot][len] + (int)(look2 >> (16 - len))) & 0xff];
  const uint32_t e2 = make_entry(true, len, sym);
  const int t2 = (int)(e2 & 31), size2 = (int)(e2 >> 5) & 15, zinc2 = (int)(e2 >> 9);
  if (t2 > room) return e1;
  return (uint32_t)(t1 + t2) | ((uint32_t)size1 << 5) | ((uint32_t)min(zinc1 + zinc2, 127) << 9) |
         ((uint32_t)t1 << 16) | ((uint32_t)size2 << 21) | ((uint32_t)zinc1 << 25);
}

// inf = sinfo of the table: [0:5) 32 - first-level bits, [5:21) LUT byte
// offset, [21:24) slot, [24:27) second-level set, [27:31) first-level bits.
// The first-level index is the top bits of the reader's high word, one
// shift by the low field (the shifter reads 5 bits).  A slot without a
// first-level LUT (bits 0) has shift 31 onto two reserved zero words.
// Write-pass reader: every step issues exactly one buffer load (a lane that
// does not refill reads out of range: no access, returns 0) and the step
// then issues exactly three buffer stores (out of range when a lane has
// nothing to store).  vmcnt counts loads and stores in issue order, so with
// these static counts the next step waits for its load with vmcnt(3) instead
// of draining the previous steps' coefficient stores (vmcnt(0), which the
// conditional global stores forced).
// (BUF_OOR / BUF_CFG: device_common.h)
struct BufReader {
  __amdgpu_buffer_rsrc_t rs;
  uint64_t acc;
  int nb;
  uint32_t wo;  // byte offset of the word in nxt
  uint32_t nxt, ld;
  bool rp;  // the previous step refilled: its load (ld) is the next word
  FFCV_DEV uint32_t word(uint32_t off) const { return __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0); }
  FFCV_DEV void init(const uint32_t *words, uint32_t nbytes, uint32_t p) {
    rs = __builtin_amdgcn_make_buffer_rsrc((void *)words, 0, (int)nbytes, BUF_CFG);
    wo = (p >> 5) * 4;
    const uint32_t w0 = __builtin_bswap32(word(wo)), w1 = __builtin_bswap32(word(wo + 4));
    wo += 8;
    nxt = word(wo);
    ld = 0;
    rp = false;
    acc = (((uint64_t)w0 << 32) | (uint64_t)w1) << (p & 31);
    nb = 64 - (int)(p & 31);
  }
  FFCV_DEV void begin() { nxt = rp ? ld : nxt; }
  FFCV_DEV void consume(int n) {
    acc <<= n;
    nb -= n;
    const bool r = nb <= 32;
    acc |= r ? (uint64_t)__builtin_bswap32(nxt) << (r ? 32 - nb : 0) : 0ull;
    nb += r ? 32 : 0;
    wo += r ? 4u : 0u;
    ld = word(r ? wo : BUF_OOR);
    rp = r;
  }
};

FFCV_DEV uint32_t si_pack(uint32_t base, uint32_t bits, uint32_t slot, uint32_t set) {
  return (bits ? 32 - bits : 31) | (base * 4) << 5 | slot << 21 | set << 24 | bits << 27;
}
FFCV_DEV uint32_t si_base(uint32_t inf) { return ((inf >> 5) & 0xffff) >> 2; }
FFCV_DEV int si_bits(uint32_t inf) { return (int)(inf >> 27) & 15; }
FFCV_DEV int si_set(uint32_t inf) { return (int)(inf >> 24) & 7; }

template <class TB>
FFCV_DEV uint32_t decode_entry(const TB &T, uint32_t acmask, uint32_t inf, uint64_t acc, bool live = true) {
  const uint32_t hi = (uint32_t)(acc >> 32);
  uint32_t e = *(const uint32_t *)((const uint8_t *)T.lut + ((inf >> 5) & 0xffff) + ((hi >> (inf & 31)) << 2));
  if ((e & 31) == 0 && live) {  // (a finished lane of a wave-uniform loop skips the rare paths)
    const uint32_t look = hi >> 16;
    const int bits = si_bits(inf), slot = (int)(inf >> 21) & 7;
    if (e) e = T.lut2[si_set(inf)][(e >> 5) - 1][(look >> (16 - bits - SUBB)) & ((1 << SUBB) - 1)];
    if ((e & 31) == 0) e = slow_entry(T, acmask, slot, look);
  }
  return e;
}

FFCV_DEV int slot_of(uint32_t pack, int ph) { return (int)((pack >> (3 * ph)) & 7); }

// SYNC decode of a lane's range [st.pos, end_bit): counts the blocks started
// in it and records their start events (the first NEV; row NEV is a dummy
// that absorbs every non-recording store).  With use_old (a later round) it
// stops at a block start that matches an event of the lane's previous
// trajectory and splices onto it: from an identical state the old trajectory
// is exact, so its remaining count and exit state are reused.  A splice off
// the new trajectory's slot grid keeps the old events from the hit on, on a
// grid based at the hit's block count (eb), when they outnumber the new ones:
// a lane re-run again in a later round then still finds them (the sync
// rounds' wave-iterations fell 808 -> 774 per image, round 4).  The old-event
// cursor advances one event per symbol (old events behind the decode
// position can never match); lagging only delays a splice, never makes a
// wrong one.  Events are double-buffered: buffer cb holds the previous
// trajectory's, cb ^ 1 receives the new one.
//
// The loop body is straight-line except the refill, the second-level lookup
// and the canonical fallback: with 64 lanes some lane starts or ends a block
// on almost every step, so those updates are selects fed by loads issued at
// the top of the step (next phase's table infos, next old event).
template <bool use_old, class TB>
FFCV_DEV DecState sync_range(JShared &S, const TB &T, const uint32_t *words, DecState st,
                             uint32_t end_bit, int lane, uint32_t &cnt, int &nev, int &cb, int &eb,
                             DecState old_exit, int sh, uint32_t &iters) {
  const int smask = (1 << sh) - 1;  // events: every 2^sh-th block start (slot q = block eb + (q << sh))
  BitReader br;
  br.init(words, st.pos);
  uint32_t pos = st.pos;
  int z = st.z, ph = st.ph;
  uint32_t dinf = S.phr[ph].dinf, ainf = S.phr[ph].ainf;
  int nph = S.phr[ph].next;
  const int ob = cb, nbuf = cb ^ 1;
  const int onev = use_old ? nev : 0;
  const uint32_t *evo = &S.ev[ob][0][lane];
  uint32_t *evn = &S.ev[nbuf][0][lane];
  int j = 0;
  uint32_t ocur = onev > 0 ? evo[0] : 0xFFFFFFFFu;
  int n = 0;
  bool hit = false;
  while (pos < end_bit && !hit) {
    K1_DIAG(iters++);
    const uint32_t ndinf = S.phr[nph].dinf, nainf = S.phr[nph].ainf;
    const int nnph = S.phr[nph].next;
    const bool isblk = z == 0;
    const uint32_t key = (pos << 4) | (uint32_t)ph;
    if constexpr (use_old) {
      const uint32_t onext = evo[min(j + 1, NEV) * JL];
      hit = isblk && ocur == key;
      const bool adv = ocur < key;
      j += adv ? 1 : 0;
      ocur = adv ? (j < onev ? onext : 0xFFFFFFFFu) : ocur;
    }
    const bool rec = isblk && !hit;
    // slot n >> sh at a block start on the slot grid, else the dummy row NEV:
    // nz is 0 exactly then, and any non-zero nz pushes the index past NEV.
    // (A hit step may write its key: the splice below copies that same old
    // event into that slot.)
    const uint32_t nz = ((uint32_t)n & (uint32_t)smask) | (uint32_t)z;
    evn[min((n >> sh) + (int)(nz << 8), NEV) * JL] = key;
    n += rec ? 1 : 0;
    const uint32_t e = decode_entry(T, S.acmask, isblk ? dinf : ainf, br.acc);
    // a pair whose first symbol ends the block decodes that symbol alone
    // (e >> 16: its bits and advance); a hit leaves the loop, its step unused
    const uint32_t v = z + (int)(e >> 25) >= 64 ? e >> 16 : e;
    const int nbits = (int)(v & 31);
    br.consume(nbits);
    pos += nbits;
    z += (int)(v >> 9) & 127;
    const bool bend = z >= 64;
    z = bend ? 0 : z;
    ph = bend ? nph : ph;
    nph = bend ? nnph : nph;
    dinf = bend ? ndinf : dinf;
    ainf = bend ? nainf : ainf;
  }
  if (hit) {  // at the previous trajectory's event j = its block start eb + (j << sh)
    const uint32_t ocnt = (uint32_t)eb + ((uint32_t)j << sh);
    int m = min((n + smask) >> sh, NEV);  // slots written so far
    if ((n & smask) == 0 && m < NEV) {     // the old events stay on the slot grid: keep them
      const int keep = min(onev - j, NEV - m);
      for (int q = 0; q < keep; q++) evn[(m + q) * JL] = evo[(j + q) * JL];
      m += keep;
      eb = 0;
    } else if (onev - j > m) {  // off the grid: the old events from j on, on a grid based at n
      const int keep = min(onev - j, NEV);
      for (int q = 0; q < keep; q++) evn[q * JL] = evo[(j + q) * JL];
      m = keep;
      eb = n;
    } else {
      eb = 0;
    }
    nev = m;
    cnt = (uint32_t)n + (cnt - ocnt);
    cb = nbuf;
    return old_exit;
  }
  nev = min((n + smask) >> sh, NEV);
  cnt = (uint32_t)n;
  eb = 0;
  cb = nbuf;
  DecState out;
  out.pos = pos;
  out.z = z;
  out.ph = ph;
  return out;
}

// WRITE decode: DC differences of every block and the AC coefficients (in
// zigzag order; the IDCT de-zigzags in registers) of the blocks inside the
// window.  blk = index of the block in progress (z > 0) or of the next block
// to start (z == 0).  Straight-line like sync_range: the next block's
// destination and window test are computed from the next phase's
// descriptor (loaded at the top of the step) and selected at a block end.
FFCV_DEV void locate_block(const int4 pd0, const int4 pd1, uint32_t blk, uint32_t nblocks, int mx, int my,
                           uint32_t &boff, bool &inwin) {
  // pd0 = {base block, blocks per MCU row, hs, mx_lo}, pd1 = {mx_hi, my_lo, my_hi, component}
  inwin = blk < nblocks && mx >= pd0.w && mx <= pd1.x && my >= pd1.y && my <= pd1.z;
  boff = ((uint32_t)pd0.x + __umul24((uint32_t)my, (uint32_t)pd0.y) + __umul24((uint32_t)mx, (uint32_t)pd0.z)) * 64u;
}

// jdhuff.c HUFF_EXTEND of the s extra bits at bit offset off of w (from
// the LSB): branch-free, 0 for s = 0.
FFCV_DEV int huff_value(uint32_t w, uint32_t off, uint32_t s) {
  const uint32_t raw = __builtin_amdgcn_ubfe(w, off, s), msb = __builtin_amdgcn_ubfe(w, off + s - 1, 1);
  return (int)(msb ? raw : raw - ((1u << s) - 1u));
}

typedef __attribute__((address_space(1))) int16_t gshort_t;  // global memory
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// Coefficient stores.  A 2-byte store per non-zero coefficient, scattered
// over the window's blocks, cost ~23% of this kernel (measured without them),
// about in proportion to the lanes that store.  So the AC coefficients at
// zigzag positions below ACS_Z (most of a block's non-zero ones) collect in
// the lane's LDS slot (the event area, dead after the sync pass) and leave as
// three 16-byte stores when the block ends; the rest, and the blocks a lane
// shares with its neighbour (the one it starts inside, the one it stops
// inside: their positions below the split belong to one lane each), are
// stored directly.  The window coefficients were zeroed before this pass, so
// unwritten positions read as zero either way.  Every step issues the same
// vector memory instructions (out-of-range offsets where a lane has nothing
// to store), so the refill waits on a static vmcnt.
template <class TB>
FFCV_DEV void write_range(JShared &S, const TB &T, const uint32_t *words, uint32_t words_bytes, DecState st,
                          uint32_t end_bit, uint32_t blk, gshort_t *coef, uint32_t coef_bytes, gshort_t *dcd,
                          uint32_t dcd_bytes, uint32_t &iters, bool dc_diffs, int &rs0, int &rs1, int &rs2) {
  uint4 *acs = S.acs[threadIdx.x % JL];
  int16_t *acs16 = (int16_t *)acs;
#pragma unroll
  for (int q = 0; q < ACS_BYTES / 16; q++) acs[q] = make_uint4(0, 0, 0, 0);
  bool stg = st.z == 0;  // a block entered part-way is the previous lane's to stage
  BufReader br;
  br.init(words, words_bytes, st.pos);
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc((void *)coef, 0, (int)coef_bytes, BUF_CFG);
  const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc((void *)dcd, 0, (int)dcd_bytes, BUF_CFG);
  uint32_t pos = st.pos;
  int z = st.z, ph = st.ph;
  const int bpm = S.bpm, mcux = S.mcux;
  const uint32_t nblocks = (uint32_t)S.nblocks;
  uint32_t dinf = S.phr[ph].dinf, ainf = S.phr[ph].ainf;
  int nph = S.phr[ph].next;
  int m = (int)(blk / bpm);
  int my = m / mcux, mx = m - my * mcux;
  uint32_t boff;
  bool inwin;
  locate_block(S.phr[ph].pd0, S.phr[ph].pd1, blk, nblocks, mx, my, boff, inwin);
  int cc = S.phr[ph].pd1.w;  // component of the block in progress
  int r0 = 0, r1 = 0, r2 = 0;  // running DC sums of the blocks this lane started
  const bool alive = true;  // (a wave-uniform loop with finished lanes idling measured neutral)
  while (pos < end_bit && !(z == 0 && blk >= nblocks)) {
    K1_DIAG(iters++);
    br.begin();
    const uint32_t ndinf = S.phr[nph].dinf, nainf = S.phr[nph].ainf;
    const int nnph = S.phr[nph].next;
    const int4 npd0 = S.phr[nph].pd0, npd1 = S.phr[nph].pd1;
    const bool isblk = z == 0 && alive;
    const uint32_t e = decode_entry(T, S.acmask, z == 0 ? dinf : ainf, br.acc, alive);
    // see make_pair: vs = this step's bits and z advance
    const int zi1 = alive ? (int)(e >> 25) : 0;
    const bool one = z + zi1 >= 64, pair = zi1 != 0;
    const uint32_t vs = alive ? (one ? e >> 16 : e) : 0u;
    const int nbits = (int)(vs & 31), zadd = (int)(vs >> 9) & 127;
    const int t1 = pair ? (int)(e >> 16) & 31 : nbits, zinc = pair ? zi1 : zadd;
    const uint32_t size = (e >> 5) & 15, size2 = pair && !one ? (e >> 21) & 15 : 0u;
    // the extra bits sit in the reader's high word (t1, nbits <= 31)
    const uint32_t hi = (uint32_t)(br.acc >> 32);
    const int v = huff_value(hi, 32 - t1, size), v2 = huff_value(hi, 32 - nbits, size2);
    br.consume(nbits);
    pos += nbits;
    // three stores every step (see BufReader): DC difference, first and
    // second AC coefficient, each out of range when the lane has none
    const uint32_t o1 = (boff + (uint32_t)min(z + zinc - 1, 63)) * 2, o2 = (boff + (uint32_t)min(z + zadd - 1, 63)) * 2;
    {  // DC: the difference itself (coefficient output) or this lane's running sum
      const int rsum = (cc == 0 ? r0 : (cc == 1 ? r1 : r2)) + v;
      r0 = isblk && cc == 0 ? rsum : r0;
      r1 = isblk && cc == 1 ? rsum : r1;
      r2 = isblk && cc == 2 ? rsum : r2;
      if (dc_diffs)
        __builtin_amdgcn_raw_buffer_store_b16((short)v, drs, isblk ? blk * 2 : BUF_OOR, 0, 0);
      else if (isblk && inwin)
        acs16[0] = (int16_t)rsum;  // a DC step starts the block: this lane stages it
    }
    const int p1 = min(z + zinc - 1, 63), p2 = min(z + zadd - 1, 63);
    const bool a1 = z != 0 && size && inwin && alive, a2 = size2 && inwin && alive;
    const bool l1 = a1 && stg && p1 < ACS_Z, l2 = a2 && stg && p2 < ACS_Z;
    if (l1) acs16[p1] = (int16_t)v;
    if (l2) acs16[p2] = (int16_t)v2;
    // (issuing these under exec masks instead measured 0.6-2% slower: K1's
    // refill would then wait for every pending store, see BufReader)
    __builtin_amdgcn_raw_buffer_store_b16((short)v, crs, a1 && !l1 ? o1 : BUF_OOR, 0, K1_CF_CPOL);
    __builtin_amdgcn_raw_buffer_store_b16((short)v2, crs, a2 && !l2 ? o2 : BUF_OOR, 0, K1_CF_CPOL);
    z += zadd;
    const bool bend = z >= 64;
    {  // a staged block that ends leaves as three 16-byte stores
      const bool fl = bend && stg && inwin;
      // left undefined where the lane does not flush (its stores go out of
      // range): zeroing it cost 12 moves per step
      uint4 c[ACS_BYTES / 16];
      if (fl) {
#pragma unroll
        for (int q = 0; q < ACS_BYTES / 16; q++) {
          c[q] = acs[q];
          acs[q] = make_uint4(0, 0, 0, 0);
        }
      }
      const uint32_t fo = fl ? boff * 2 : BUF_OOR;
#pragma unroll
      for (int q = 0; q < ACS_BYTES / 16; q++)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, c[q]), crs, fo + 16 * q, 0, K1_CF_CPOL);
    }
    stg = stg || bend;
    // the next block: (blk + 1, nph, mx', my')
    const bool wrap = nph == 0;
    const int nmx = wrap ? (mx + 1 == mcux ? 0 : mx + 1) : mx;
    const int nmy = wrap && mx + 1 == mcux ? my + 1 : my;
    uint32_t nboff;
    bool ninwin;
    locate_block(npd0, npd1, blk + 1, nblocks, nmx, nmy, nboff, ninwin);
    z = bend ? 0 : z;
    blk += bend ? 1 : 0;
    ph = bend ? nph : ph;
    nph = bend ? nnph : nph;
    mx = bend ? nmx : mx;
    my = bend ? nmy : my;
    dinf = bend ? ndinf : dinf;
    ainf = bend ? nainf : ainf;
    boff = bend ? nboff : boff;
    inwin = bend ? ninwin : inwin;
    cc = bend ? npd1.w : cc;
  }
  rs0 = r0;
  rs1 = r1;
  rs2 = r2;
  if (stg && z > 0 && inwin) {  // stopped inside a staged block: its positions below z are this lane's
    for (int q = 0; q < ACS_Z; q++) {
      const int c = acs16[q];
      if (q < z && c != 0) __builtin_amdgcn_raw_buffer_store_b16((short)c, crs, (boff + (uint32_t)q) * 2, 0, K1_CF_CPOL);
    }
  }
}

// Cross-lane helpers on DPP (no LDS round trip, unlike __shfl's
// ds_bpermute).  All lanes of the wave must be active.
//   wave_exscan: exclusive prefix sum (row_shr 1/2/4/8, row_bcast 15/31)
//   lane_prev / lane_next: value of lane t-1 / t+1 (0 past the ends)
FFCV_DEV uint32_t wave_exscan(uint32_t v) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  return (uint32_t)x - v;
}
FFCV_DEV uint32_t lane_prev(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false); }
FFCV_DEV uint32_t lane_next(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false); }
FFCV_DEV uint32_t lane_read(uint32_t v, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)v, lane); }
FFCV_DEV int32_t wave_exscan_i(int32_t v) { return (int32_t)wave_exscan((uint32_t)v); }

// The same over the JL-lane segments of a wave (one image each); t = lane in
// the segment, sg = segment.  Cross-segment DPP sources are masked off.
FFCV_DEV uint32_t seg_exscan(uint32_t v) {
  if constexpr (JL == JT) return wave_exscan(v);
  int x = (int)v;  // row_shr 1/2/4/8 within 16-lane rows, then row_bcast 15 into rows 1 and 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  return (uint32_t)x - v;
}
FFCV_DEV int32_t seg_exscan_i(int32_t v) { return (int32_t)seg_exscan((uint32_t)v); }
FFCV_DEV uint32_t seg_prev(uint32_t v, int t) {
  const uint32_t p = lane_prev(v);
  return t == 0 ? 0u : p;
}
FFCV_DEV uint32_t seg_next(uint32_t v, int t) {
  const uint32_t n = lane_next(v);
  return t == JL - 1 ? 0u : n;
}
// value of lane i of this lane's segment (i uniform)
FFCV_DEV uint32_t seg_read(uint32_t v, int i, int sg) {
  if constexpr (JL == JT) return lane_read(v, i);
  const uint32_t a = lane_read(v, i), b = lane_read(v, JL + i);
  return sg ? b : a;
}
FFCV_DEV uint64_t seg_ballot(bool p, int sg) {
  const uint64_t m = __ballot(p);
  if constexpr (JL == JT) return m;
  return (m >> (JL * sg)) & ((1ull << JL) - 1);
}
FFCV_DEV bool seg_any(bool p, int sg) { return seg_ballot(p, sg) != 0; }


// libjpeg post-IDCT range limit: table[x & 1023] (jdmaster.c)
FFCV_DEV uint8_t idct_rl(int x) {
  // table[x & 1023] = x+128 (x & 1023 < 128), 255 (< 512), 0 (< 896), x-896:
  // with u = (x + 128) & 1023 that is min(u, 255) below 640, else 0
  const uint32_t u = (uint32_t)(x + 128) & 1023u;
  return (uint8_t)(u >= 640u ? 0u : min(u, 255u));
}
// jidctfst.c MULTIPLY: DESCALE(var * const, CONST_BITS = 8) with a JLONG
// (64-bit) product.  The 32-bit form is identical whenever the product fits.
// Interval bounds through jpeg_idct_ifast with every dequantised input
// |d| <= M: pass-1 outputs <= 35.83 M (+ 5 from truncation), and the largest
// product is pass 2's (z10 + z12) * 473 <= 67,787 M, below 2^31 for
// M <= 31,680 (tools/idct_bound.py); the 32-bit form is used for M <= 30,000
// and WIDE keeps the exact 64-bit form for the rest.
template <bool WIDE>
FFCV_DEV int fmul8(int v, int c) {
  return WIDE ? (int)(((int64_t)v * c) >> 8) : (v * c) >> 8;
}

// jidctfst.c jpeg_idct_ifast on one dequantised block d (natural order),
// straight-line: the reference's all-zero-AC shortcuts produce the same
// values, so they are not taken (they would only diverge the wave).
template <bool WIDE>
FFCV_DEV void idct_ifast_block(int d[64], uint8_t *out, int stride) {
#pragma unroll
  for (int c = 0; c < 8; c++) {
    int tmp0 = d[c], tmp1 = d[16 + c], tmp2 = d[32 + c], tmp3 = d[48 + c];
    int tmp10 = tmp0 + tmp2, tmp11 = tmp0 - tmp2;
    int tmp13 = tmp1 + tmp3, tmp12 = fmul8<WIDE>(tmp1 - tmp3, 362) - tmp13;
    tmp0 = tmp10 + tmp13;
    tmp3 = tmp10 - tmp13;
    tmp1 = tmp11 + tmp12;
    tmp2 = tmp11 - tmp12;
    int tmp4 = d[8 + c], tmp5 = d[24 + c], tmp6 = d[40 + c], tmp7 = d[56 + c];
    int z13 = tmp6 + tmp5, z10 = tmp6 - tmp5, z11 = tmp4 + tmp7, z12 = tmp4 - tmp7;
    tmp7 = z11 + z13;
    tmp11 = fmul8<WIDE>(z11 - z13, 362);
    int z5 = fmul8<WIDE>(z10 + z12, 473);
    tmp10 = fmul8<WIDE>(z12, 277) - z5;
    tmp12 = fmul8<WIDE>(z10, -669) + z5;
    tmp6 = tmp12 - tmp7;
    tmp5 = tmp11 - tmp6;
    tmp4 = tmp10 + tmp5;
    d[c] = tmp0 + tmp7;
    d[56 + c] = tmp0 - tmp7;
    d[8 + c] = tmp1 + tmp6;
    d[48 + c] = tmp1 - tmp6;
    d[16 + c] = tmp2 + tmp5;
    d[40 + c] = tmp2 - tmp5;
    d[32 + c] = tmp3 + tmp4;
    d[24 + c] = tmp3 - tmp4;
  }
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const int *w = d + 8 * r;
    int tmp10 = w[0] + w[4], tmp11 = w[0] - w[4];
    int tmp13 = w[2] + w[6], tmp12 = fmul8<WIDE>(w[2] - w[6], 362) - tmp13;
    int tmp0 = tmp10 + tmp13, tmp3 = tmp10 - tmp13, tmp1 = tmp11 + tmp12, tmp2 = tmp11 - tmp12;
    int z13 = w[5] + w[3], z10 = w[5] - w[3], z11 = w[1] + w[7], z12 = w[1] - w[7];
    int tmp7 = z11 + z13;
    tmp11 = fmul8<WIDE>(z11 - z13, 362);
    int z5 = fmul8<WIDE>(z10 + z12, 473);
    tmp10 = fmul8<WIDE>(z12, 277) - z5;
    tmp12 = fmul8<WIDE>(z10, -669) + z5;
    int tmp6 = tmp12 - tmp7, tmp5 = tmp11 - tmp6, tmp4 = tmp10 + tmp5;
    uint32_t o0 = idct_rl((tmp0 + tmp7) >> 5), o7 = idct_rl((tmp0 - tmp7) >> 5);
    uint32_t o1 = idct_rl((tmp1 + tmp6) >> 5), o6 = idct_rl((tmp1 - tmp6) >> 5);
    uint32_t o2 = idct_rl((tmp2 + tmp5) >> 5), o5 = idct_rl((tmp2 - tmp5) >> 5);
    uint32_t o4 = idct_rl((tmp3 + tmp4) >> 5), o3 = idct_rl((tmp3 - tmp4) >> 5);
    uint2 v;
    v.x = o0 | (o1 << 8) | (o2 << 16) | (o3 << 24);
    v.y = o4 | (o5 << 8) | (o6 << 16) | (o7 << 24);
    *(uint2 *)(out + (uint64_t)r * stride) = v;
  }
}

// One block: load the zigzag coefficients at cp, de-zigzag +
// jidctfst.c DEQUANTIZE (int16 x int16 -> int) with the multipliers qm, and
// the ifast IDCT into out (stride bytes per row).
typedef int16_t s16x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

// dc_add: added to the DC coefficient (slot 0) before dequantisation
FFCV_DEV void idct_block(const int16_t *cp, const int16_t *qm, int qmax, uint8_t *out, int stride, int dc_add) {
  int16_t zz[64];
  int d[64];
#pragma unroll
  for (int p8 = 0; p8 < 8; p8++) *(uint4 *)(zz + p8 * 8) = ((const uint4 *)cp)[p8];
  zz[0] = (int16_t)(zz[0] + dc_add);
  // max |AC coefficient| on packed halves (|-32768| reads as 32768
  // unsigned); max(|DC| * |qmul[0]|, max|AC| * max|AC qmul|) bounds every
  // dequantised input (the DC term is the large one: a bright block's DC
  // times the small DC multiplier), which selects the 32-bit IDCT products
  // when they are exact (see fmul8)
  u16x2 mu = {0, 0};
#pragma unroll
  for (int w = 0; w < 32; w++) {
    s16x2 v = *(const s16x2 *)(zz + 2 * w);
    if (w == 0) v.x = 0;  // the DC coefficient
    const s16x2 av = __builtin_elementwise_max(v, (s16x2){0, 0} - v);
    mu = __builtin_elementwise_max(mu, __builtin_bit_cast(u16x2, av));
  }
  const int cmax = max((int)mu.x, (int)mu.y);
  const int dc = zz[0], qdc = qm[0];
  const int bound = max(abs(dc) * abs(qdc), cmax * qmax);
#pragma unroll
  for (int n = 0; n < 64; n++) d[n] = (int)zz[kZigzagOfNatural[n]] * (int)qm[n];
  if (bound <= 30000)
    idct_ifast_block<false>(d, out, stride);
  else
    idct_ifast_block<true>(d, out, stride);
}

struct JpegArgs {
  const uint8_t *base;
  const ffcv_sample *samples;
  const int32_t *crops;
  const int32_t *cut;
  const uint8_t *flips;
  int32_t *crops_w;  // the same arrays, written by the fused draws
  int32_t *cut_w;
  uint8_t *flips_w;
  ffcv_rrc_params p;
  void *out;
  uint64_t out_stride;
  int32_t *status;
  // Per-launch scratch arena: K1 bump-allocates each image's regions (de-
  // stuffed stream, window coefficients, DC differences, window planes, K2
  // band staging) sized by that image's own geometry and crop window, so
  // scratch follows the content instead of dataset-max x batch.
  uint8_t *arena;
  uint64_t arena_bytes;
  unsigned long long *arena_top;  // [0] bump counter (0 when K1 starts), [1] last launch's high water
  ImgInfo *info;
  uint2 *taps;    // K2_TAPS packed linear taps per image (RRC), written by K1
  uint8_t *gtab;  // per-image JTables for images that cannot share the workgroup's
  uint64_t gtab_slot;
  int batch;
  // fused gather + draws (ffcv_jpeg_rrc_fused): samples = table[ids[k]],
  // crop / cutout / flip drawn in K1 (lanes 1-3) into crops / cut / flips
  const ffcv_sample *table;
  uint64_t n_table;
  const uint64_t *ids;
  const uint32_t *k1_order;  // K1's image of (workgroup, wave) slot i (null: i itself); see k1_order_kernel
  ffcv_sample *samples_out;
  ffcv_draw_params dp;
  int do_draw;
  uint32_t max_h, max_w;
  uint64_t max_blocks;
  uint64_t *dbg;
  int diag_only;  // host side only: kernels the launch runs (ffcv_jpeg_set_diag)
  // Entropy index (ffcv_jpeg_set_entropy_index): per dataset sample, the
  // converged start state of every lane range of the sync pass.  A sample
  // decoded once with the index attached records it; later decodes of the
  // same sample (later epochs) skip the sync rounds.  Fused launches only
  // (the sample id comes from ids[k]).
  uint32_t *eidx;
  uint64_t eidx_n;
};

// Diagnostic stamps: lane 0 records wall_clock64 at phase boundaries into
// dbg[image*16 + slot] (never read by the kernel; off when dbg == nullptr).
#define STAMP(slot)                                                          \
  do {                                                                       \
    if (a.dbg && t == 0) a.dbg[(uint64_t)k * 16 + (slot)] = wall_clock64();  \
  } while (0)

// A wave-uniform value in a scalar register (one image per wave).
FFCV_DEV uint32_t wuni(uint32_t v) {
  if constexpr (JL == JT) return __builtin_amdgcn_readfirstlane(v);
  return v;
}

// P0: marker walk over the LDS copy of the header bytes.  With one image per
// wave every lane runs it on wave-uniform (scalar) values: each byte read is
// broadcast to a scalar register, so the walk's branches and arithmetic are
// scalar instead of one lane under an exec mask.
// x / d for x >= 0 and a sampling factor or ratio d in 1..4 (the parse
// rejects anything else): shifts, or a multiply-high for 3, instead of a
// ~25-instruction VALU division sequence (the operands are wave-uniform, so
// these stay on the scalar unit)
FFCV_DEV int dsmall(int x, int d) {
  return d == 3 ? (int)(((uint64_t)(uint32_t)x * 0xAAAAAAABull) >> 33) : x >> (d >> 1);
}

FFCV_DEV int parse_header(JShared &S, const uint8_t *src, uint32_t nbytes, const ffcv_sample &smp_in,
                          const JpegArgs &a, int k_in, int MODE) {
  nbytes = wuni(nbytes);
  const int k = (int)wuni((uint32_t)k_in);
  ffcv_sample smp = smp_in;
  smp.width = wuni(smp_in.width);
  smp.height = wuni(smp_in.height);
  // (p through readfirstlane: the compiler kept the walk's position in a
  // 64-bit vector register pair and branched on it under exec masks, ~20
  // VALU per byte read; uniform, the branch and the address are scalar)
  auto B = [&](uint32_t p) -> int {
    p = wuni(p);
    int v;
    if (p < HDR_BYTES)
      v = S.hdr[p];
    else
      v = gld_u8(src + p);
    return (int)wuni((uint32_t)v);
  };
  auto R16 = [&](uint32_t p) -> int { return (B(p) << 8) | B(p + 1); };
  for (int i = 0; i < 4; i++) S.dqt_ok[i] = 0;
  for (int i = 0; i < NTAB; i++) S.dht_ok[i] = 0;
  S.saw_jfif = S.saw_adobe = 0;
  S.adobe_transform = 1;
  S.restart = 0;
  S.ncomp = 0;
  int have_sof = 0, have_sos = 0;
  if (nbytes < 4 || B(0) != 0xFF || B(1) != 0xD8) return FFCV_SAMPLE_BAD_MARKER;
  uint32_t p = 2;
  while (!have_sos) {
    p = wuni(p);
    if (p + 4 > nbytes || B(p) != 0xFF) return FFCV_SAMPLE_BAD_MARKER;
    while (p < nbytes && B(p) == 0xFF) p++;
    if (p >= nbytes) return FFCV_SAMPLE_BAD_MARKER;
    int m = B(p++);
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9 || p + 2 > nbytes) return FFCV_SAMPLE_BAD_MARKER;
    int len = R16(p);
    if (len < 2 || p + (uint32_t)len > nbytes) return FFCV_SAMPLE_BAD_MARKER;
    uint32_t s = p + 2;
    int sl = len - 2;
    if (m == 0xDB) {
      int o = 0;
      while (o < sl) {
        int pq = B(s + o) >> 4, tq = B(s + o) & 15;
        if (tq > 3) return FFCV_SAMPLE_BAD_MARKER;
        S.dqt_off[tq] = s + o + 1;
        S.dqt_prec[tq] = pq;
        S.dqt_ok[tq] = 1;
        o += 1 + (pq ? 128 : 64);
      }
    } else if (m == 0xC4) {
      int o = 0;
      while (o < sl) {
        int tc = B(s + o) >> 4, th = B(s + o) & 15;
        if (th > 3 || tc > 1) return FFCV_SAMPLE_BAD_MARKER;
        int total = 0;
        for (int l = 0; l < 16; l++) total += B(s + o + 1 + l);
        if (total > 256) return FFCV_SAMPLE_BAD_MARKER;
        S.dht_off[tc * 4 + th] = s + o + 1;
        S.dht_ok[tc * 4 + th] = 1;
        o += 17 + total;
      }
    } else if (m == 0xC0 || m == 0xC1) {
      if (B(s) != 8) return FFCV_SAMPLE_UNSUPPORTED;
      S.H = R16(s + 1);
      S.W = R16(s + 3);
      S.ncomp = B(s + 5);
      if (S.ncomp != 1 && S.ncomp != 3) return FFCV_SAMPLE_UNSUPPORTED;
      S.hmax = S.vmax = 1;
      for (int c = 0; c < S.ncomp; c++) {
        S.cid[c] = B(s + 6 + 3 * c);
        S.hs[c] = B(s + 7 + 3 * c) >> 4;
        S.vs[c] = B(s + 7 + 3 * c) & 15;
        S.tq[c] = B(s + 8 + 3 * c) & 3;
        if (S.hs[c] < 1 || S.hs[c] > 4 || S.vs[c] < 1 || S.vs[c] > 4) return FFCV_SAMPLE_UNSUPPORTED;
        S.hmax = max(S.hmax, S.hs[c]);
        S.vmax = max(S.vmax, S.vs[c]);
      }
      have_sof = 1;
    } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return FFCV_SAMPLE_UNSUPPORTED;  // progressive / lossless / arithmetic
    } else if (m == 0xDD) {
      S.restart = R16(s);
    } else if (m == 0xE0) {
      if (sl >= 5 && B(s) == 'J' && B(s + 1) == 'F' && B(s + 2) == 'I' && B(s + 3) == 'F' && B(s + 4) == 0)
        S.saw_jfif = 1;
    } else if (m == 0xEE) {
      if (sl >= 12 && B(s) == 'A' && B(s + 1) == 'd' && B(s + 2) == 'o' && B(s + 3) == 'b' && B(s + 4) == 'e') {
        S.saw_adobe = 1;
        S.adobe_transform = B(s + 11);
      }
    } else if (m == 0xDA) {
      if (!have_sof) return FFCV_SAMPLE_BAD_MARKER;
      int ns = B(s);
      if (ns != S.ncomp) return FFCV_SAMPLE_UNSUPPORTED;  // multi-scan sequential
      int order[3];
      for (int i = 0; i < ns; i++) {
        int c = -1;
        for (int q = 0; q < S.ncomp; q++)
          if (S.cid[q] == B(s + 1 + 2 * i)) c = q;
        if (c < 0) return FFCV_SAMPLE_BAD_MARKER;
        order[i] = c;
        S.td[c] = B(s + 2 + 2 * i) >> 4;
        S.ta[c] = B(s + 2 + 2 * i) & 15;
        if (S.td[c] > 3 || S.ta[c] > 3) return FFCV_SAMPLE_BAD_MARKER;
      }
      int nb = 0;
      if (S.ncomp == 1) {
        S.blk_comp[0] = order[0];
        S.blk_dx[0] = S.blk_dy[0] = 0;
        nb = 1;
      } else {
        for (int i = 0; i < ns; i++) {
          int c = order[i];
          for (int yy = 0; yy < S.vs[c]; yy++)
            for (int xx = 0; xx < S.hs[c]; xx++) {
              if (nb < 10) {
                S.blk_comp[nb] = c;
                S.blk_dx[nb] = xx;
                S.blk_dy[nb] = yy;
              }
              nb++;
            }
        }
      }
      if (nb > 10) return FFCV_SAMPLE_UNSUPPORTED;
      S.bpm = nb;
      // table slots: AC tables first (they decode most symbols), so they
      // always get a fast LUT
      S.nslots = 0;
      S.dcpack = S.acpack = S.acmask = 0;
      for (int pass = 0; pass < 2; pass++) {
        for (int b = 0; b < nb; b++) {
          int c = S.blk_comp[b];
          int tab = pass == 0 ? 4 + S.ta[c] : S.td[c];
          int sl = -1;
          for (int q = 0; q < S.nslots; q++)
            if (S.slot_tab[q] == tab) sl = q;
          if (sl < 0) {
            sl = S.nslots++;
            S.slot_tab[sl] = tab;
            if (pass == 0) S.acmask |= 1u << sl;
          }
          if (pass == 0)
            S.acpack |= (uint32_t)sl << (3 * b);
          else
            S.dcpack |= (uint32_t)sl << (3 * b);
        }
      }
      // first-level LUT space from the pool, in slot order (AC slots first)
      uint32_t used = 0, nset = 0, nac = 0;
      for (int q = 0; q < S.nslots; q++) {
        uint32_t bits = S.slot_tab[q] >= 4 ? (nac++ ? FB_AC2 : FB_AC) : FB_DC;
        if (used + (1u << bits) > LUT_POOL - 2 || nset == NLUTSLOT) bits = 0;  // canonical decode only
        S.sinfo[q] = si_pack(bits ? used : (uint32_t)(LUT_POOL - 2), bits, (uint32_t)q, bits ? nset : 0u);
        used += bits ? (1u << bits) : 0u;
        nset += bits ? 1u : 0u;
      }
      for (int b = 0; b < nb; b++) {
        S.phr[b].dinf = S.sinfo[slot_of(S.dcpack, b)];
        S.phr[b].ainf = S.sinfo[slot_of(S.acpack, b)];
        S.phr[b].next = b + 1 == nb ? 0 : b + 1;
      }
      S.scan_off = p + (uint32_t)len;
      have_sos = 1;
    }
    p += (uint32_t)len;
  }
  if (S.restart) return FFCV_SAMPLE_UNSUPPORTED;
  if (S.W != (int)smp.width || S.H != (int)smp.height) return FFCV_SAMPLE_GEOMETRY;
  if ((uint32_t)S.W > a.max_w || (uint32_t)S.H > a.max_h) return FFCV_SAMPLE_TOO_LARGE;
  for (int c = 0; c < S.ncomp; c++) {
    if (!S.dqt_ok[S.tq[c]] || !S.dht_ok[S.td[c]] || !S.dht_ok[4 + S.ta[c]]) return FFCV_SAMPLE_BAD_MARKER;
    if (S.hmax % S.hs[c] || S.vmax % S.vs[c]) return FFCV_SAMPLE_UNSUPPORTED;
  }
  if (S.ncomp == 3) {  // jdapimin.c default_decompress_parms colour-space rule
    if (S.saw_jfif)
      S.color_rgb = 0;
    else if (S.saw_adobe)
      S.color_rgb = S.adobe_transform == 0;
    else
      S.color_rgb = S.cid[0] == 82 && S.cid[1] == 71 && S.cid[2] == 66;
  } else {
    S.color_rgb = 0;
  }
  if (S.ncomp == 1) {
    S.cw[0] = dsmall(S.W * S.hs[0] + S.hmax - 1, S.hmax);
    S.ch[0] = dsmall(S.H * S.vs[0] + S.vmax - 1, S.vmax);
    S.mcux = (S.cw[0] + 7) / 8;
    S.mcuy = (S.ch[0] + 7) / 8;
    S.bw[0] = S.mcux;
    S.bh[0] = S.mcuy;
    S.hs[0] = S.vs[0] = 1;  // non-interleaved scan: one block per MCU
    S.hmax = S.vmax = 1;
  } else {
    S.mcux = dsmall((S.W + 8 * S.hmax - 1) >> 3, S.hmax);
    S.mcuy = dsmall((S.H + 8 * S.vmax - 1) >> 3, S.vmax);
    for (int c = 0; c < S.ncomp; c++) {
      S.cw[c] = dsmall(S.W * S.hs[c] + S.hmax - 1, S.hmax);
      S.ch[c] = dsmall(S.H * S.vs[c] + S.vmax - 1, S.vmax);
      S.bw[c] = S.mcux * S.hs[c];
      S.bh[c] = S.mcuy * S.vs[c];
    }
  }
  S.nblocks = S.mcux * S.mcuy * S.bpm;
  if (MODE == JM_COEF && (uint64_t)S.nblocks > a.max_blocks) return FFCV_SAMPLE_TOO_LARGE;
  if (MODE == JM_RRC) {
    // vector loads (the fused draws wrote the crop with vector stores in this
    // kernel; a scalar load at this uniform address could hit a stale K$ line)
    auto crop = [&](int i) {
      return (int)wuni((uint32_t)__builtin_nontemporal_load((const __attribute__((address_space(1))) int32_t *)a.crops + 4 * k + i));
    };
    S.ri = crop(0);
    S.rj = crop(1);
    S.rh = crop(2);
    S.rw = crop(3);
    if (S.rh <= 0 || S.rw <= 0 || S.ri < 0 || S.rj < 0 || S.ri + S.rh > S.H || S.rj + S.rw > S.W)
      return FFCV_SAMPLE_GEOMETRY;
  } else {
    S.ri = 0;
    S.rj = 0;
    S.rh = S.H;
    S.rw = S.W;
  }
  for (int c = 0; c < S.ncomp; c++) {  // blocks the crop reads (+1 sample of fancy context)
    int he = dsmall(S.hmax, S.hs[c]), ve = dsmall(S.vmax, S.vs[c]);
    int y0 = dsmall(S.ri, ve) - (ve == 2 ? 1 : 0), y1 = dsmall(S.ri + S.rh - 1, ve) + (ve == 2 ? 1 : 0);
    int x0 = dsmall(S.rj, he) - (he == 2 ? 1 : 0), x1 = dsmall(S.rj + S.rw - 1, he) + (he == 2 ? 1 : 0);
    y0 = max(y0, 0);
    x0 = max(x0, 0);
    y1 = min(y1, S.ch[c] - 1);
    x1 = min(x1, S.cw[c] - 1);
    if (MODE == JM_COEF) {
      y0 = x0 = 0;
      y1 = S.bh[c] * 8 - 1;
      x1 = S.bw[c] * 8 - 1;
    }
    S.wy0[c] = y0 >> 3;
    S.wy1[c] = y1 >> 3;
    S.wx0[c] = x0 >> 3;
    S.wx1[c] = x1 >> 3;
  }
  uint32_t nwin = 0;  // coefficients / planes are stored for the window only
  for (int c = 0; c < S.ncomp; c++) {
    S.coff[c] = nwin;
    nwin += (uint32_t)((S.wx1[c] - S.wx0[c] + 1) * (S.wy1[c] - S.wy0[c] + 1));
  }
  S.nwin = nwin;
  for (int b = 0; b < S.bpm; b++) {
    int c = S.blk_comp[b], dx = S.blk_dx[b], dy = S.blk_dy[b], hs = S.hs[c], vs = S.vs[c];
    // bx = mx * hs + dx in [wx0, wx1]  <=>  mx in [mx_lo, mx_hi]
    int mxl = S.wx0[c] - dx <= 0 ? 0 : dsmall(S.wx0[c] - dx + hs - 1, hs);
    int mxh = S.wx1[c] - dx < 0 ? -1 : dsmall(S.wx1[c] - dx, hs);
    int myl = S.wy0[c] - dy <= 0 ? 0 : dsmall(S.wy0[c] - dy + vs - 1, vs);
    int myh = S.wy1[c] - dy < 0 ? -1 : dsmall(S.wy1[c] - dy, vs);
    // window-relative index of block (mx * hs + dx, my * vs + dy) is
    // base + my * (vs * wbw) + mx * hs (base may be negative: only window
    // blocks are ever addressed, and the sum wraps back in 32 bits)
    const int wbw = S.wx1[c] - S.wx0[c] + 1;
    S.phr[b].pd0 = make_int4((int)S.coff[c] + (dy - S.wy0[c]) * wbw + (dx - S.wx0[c]), vs * wbw, hs, mxl);
    S.phr[b].pd1 = make_int4(mxh, myl, myh, c);  // .w: the phase's component (write pass DC sums)
  }
  return FFCV_SAMPLE_OK;
}

// Wave-level syncs: K1's waves decode independent images, so after the
// workgroup's shared table build each wave orders only its own lanes.
FFCV_DEV void wsync_lds() {  // LDS writes of this wave visible to its lanes
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
FFCV_DEV void wsync_mem() {  // LDS and global writes of this wave visible to its lanes
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
}

// P1: Huffman decode tables for the table slots of image R (jdhuff.c
// jpeg_make_d_derived_tbl, including its table checks), by NT threads: the
// workgroup into its shared LDS copy, or one wave into its own global copy.
template <int NT, class TB, class HBF>
FFCV_DEV void build_tables(TB &T, const JShared &R, const HBF &HB, int tid) {
  auto bar = [&]() {
    if constexpr (NT == JL)
      wsync_mem();
    else
      __syncthreads();
  };
  const int nslots = R.nslots;
  if (tid == 0) T.bad = 0;
  bar();
  if (tid < nslots) {
    const int tab = R.slot_tab[tid];
    const uint32_t d = R.dht_off[tab];
    uint32_t code = 0;
    int kk = 0;
    bool bad = false;
    for (int l = 1; l <= 16; l++) {
      int nl = HB(d + l - 1);
      T.valoff[tid][l] = kk - (int)code;
      code += nl;
      kk += nl;
      if (code >= (1u << l)) bad = true;  // over-subscribed (or all-ones) code space
      T.lim[tid][l] = code << (16 - l);
      code <<= 1;
    }
    T.nvals[tid] = kk;
    if (bad) T.bad = 1;
    T.nsub[tid] = 0;
  }
  bar();
  for (int s2 = 0; s2 < nslots; s2++) {
    const int tab = R.slot_tab[s2];
    const uint32_t d = R.dht_off[tab];
    for (int i = tid; i < T.nvals[s2]; i += NT) {
      int v = HB(d + 16 + i);
      if (tab < 4 && v > 15) T.bad = 1;  // DC sizes are 0..15
      T.vals[s2][i] = (uint8_t)v;
    }
  }
  if (tid < 2) T.lut[LUT_POOL - 2 + tid] = 0;  // the zero words of LUT-less slots
  bar();
  for (int s = 0; s < nslots; s++) {
    const uint32_t inf = R.sinfo[s];
    const int bits = si_bits(inf);
    if (!bits) continue;
    const bool ac = (R.acmask >> s) & 1;
    uint32_t L[FB_AC + 1];
#pragma unroll
    for (int l = 1; l <= FB_AC; l++) L[l] = T.lim[s][l];
    for (int v = tid; v < (1 << bits); v += NT) {
      const uint32_t look = (uint32_t)v << (16 - bits);
      int len = 1;
#pragma unroll
      for (int l = 1; l < FB_AC; l++) len += (l < bits && look >= L[l]) ? 1 : 0;
      uint32_t e = 0;
      if (look < T.lim[s][len]) {
        int sym = T.vals[s][(T.valoff[s][len] + (int)(look >> (16 - len))) & 0xff];
        e = make_entry(ac, len, sym);
      } else if (look < T.lim[s][16]) {  // codes longer than `bits` under this prefix
        int n = atomicAdd(&T.nsub[s], 1);
        if (n < NSUB) {
          T.sub_prefix[s][n] = (uint16_t)v;
          e = (uint32_t)(n + 1) << 5;
        }
      }
      if (ac && e) e = make_pair(T, s, bits, L, look, e);
      T.lut[si_base(inf) + v] = e;
    }
  }
  bar();
  for (int i = tid; i < NSLOT * NSUB * (1 << SUBB); i += NT) {
    const int s = i / (NSUB << SUBB), n = (i >> SUBB) % NSUB, x = i & ((1 << SUBB) - 1);
    if (s >= nslots || n >= min(T.nsub[s], NSUB)) continue;
    const int bits = si_bits(R.sinfo[s]);
    const uint32_t look = ((uint32_t)T.sub_prefix[s][n] << (16 - bits)) | ((uint32_t)x << (16 - bits - SUBB));
    int len = 1;
    for (int l = 1; l < 16; l++) len += look >= T.lim[s][l];
    T.lut2[si_set(R.sinfo[s])][n][x] = len <= bits + SUBB ? (uint16_t)slow_entry(T, R.acmask, s, look) : (uint16_t)0;
  }
  bar();
}

// P3-P5 with table set T (the workgroup's LDS copy or the image's global
// copy; separate instantiations so each reads its own address space).
// Entropy index record of one sample: EIDX_WORDS words per lane range t >= 1,
// [pos, z | ph << 8, first block].  Lane 0's range always starts at (0, 0, 0),
// so its words carry [hash high, EIDX_VALID | nthr << 16, hash low]: a 64-bit
// hash of the other lanes' words.  Records are written and read with plain
// memory operations and no fences (an agent-scope release / acquire writes
// back / invalidates the whole L2 of the XCD): a record is used only when its
// hash matches, so a reader that sees part of a record being published by a
// concurrent launch on another XCD (lines not yet written back) decodes the
// sample in full instead.  A record's content is a pure function of the
// sample, so every publish writes the same words.
#define EIDX_LANES 64
#define EIDX_WORDS 3
#define EIDX_VALID 0x80000000u
FFCV_DEV uint64_t eidx_hash(uint32_t w0, uint32_t w1, uint32_t w2, int t) {
  // per lane mix, then an xor over the wave (wave-uniform result)
  uint64_t h = ((uint64_t)w0 << 32 | w1) * 0x9E3779B97F4A7C15ull ^ ((uint64_t)w2 << 32 | (uint32_t)t) * 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 29;
  uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    lo ^= (uint32_t)__shfl_xor((int)lo, m);
    hi ^= (uint32_t)__shfl_xor((int)hi, m);
  }
  return ((uint64_t)hi << 32) | lo;
}
// Zero the image's window coefficients right before the write pass stores
// its non-zero ones: the lines are then still in L2 when the scattered 2-byte
// stores and the IDCT's block reads reach them (zeroed at allocation, ~300 us
// earlier, they had been written back and the stores missed).
FFCV_DEV void zero_window_coefs(const JShared &S, int16_t *coef, int t) {
#ifdef K1_NOZERO
  return;  // diagnostics (wrong pixels): the zeroing's share of K1's traffic and time
#endif
  // (buffer stores: no flat_store, which would also count in lgkmcnt)
  const __amdgpu_buffer_rsrc_t zrs =
      __builtin_amdgcn_make_buffer_rsrc(wave_uniform((void *)coef), 0, (int)wuni(S.cf_bytes), BUF_CFG);
  const uint32_t n = wuni((uint32_t)(S.nwin * 8));
  for (uint32_t i = (uint32_t)t; i < n; i += JL)
    __builtin_amdgcn_raw_buffer_store_b128((u32x4_t){0u, 0u, 0u, 0u}, zrs, 16 * i, 0, K1_CF_CPOL);
  wsync_mem();
}

template <class TB>
FFCV_DEV bool entropy_passes(JShared &S, const TB &T, const JpegArgs &a, int k, int t, int sg, const uint32_t *words,
                             uint32_t total_bits, int16_t *coef, int16_t *dcd, uint64_t sample_id, bool dc_diffs) {
  int rs0 = 0, rs1 = 0, rs2 = 0;
  uint32_t start_blk = 0;  // first block this lane starts
  // each lane's DC offsets and start block for jpeg_idct_kernel (non-coefficient modes)
  auto publish_dc = [&]() {
    if (dc_diffs) return;
    const int o0 = seg_exscan_i(rs0), o1 = seg_exscan_i(rs1), o2 = seg_exscan_i(rs2);
    ImgInfo *info = a.info + k;
    info->lane_blk0[t] = start_blk;
    info->lane_off[0][t] = o0;
    info->lane_off[1][t] = o1;
    info->lane_off[2][t] = o2;
  };
  uint32_t nthr = (total_bits + 191) / 192;
  nthr = max(1u, min(nthr, (uint32_t)JL));
  const uint32_t cbits = (total_bits + nthr - 1) / nthr;
  const bool active = t < (int)nthr;
  const uint32_t my_end = active ? (t == (int)nthr - 1 ? total_bits : min(total_bits, (t + 1) * cbits)) : 0;
  // ---------------------------------------------------- entropy index ----
  uint32_t *rec = nullptr;
  if (a.eidx && JL == EIDX_LANES && sample_id < a.eidx_n) rec = a.eidx + sample_id * (EIDX_LANES * EIDX_WORDS);
  if (rec) {
    const uint32_t w0 = __builtin_nontemporal_load(rec + EIDX_WORDS * t);
    const uint32_t w1 = __builtin_nontemporal_load(rec + EIDX_WORDS * t + 1);
    const uint32_t w2 = __builtin_nontemporal_load(rec + EIDX_WORDS * t + 2);
    const uint32_t head = __builtin_amdgcn_readfirstlane(w1);
    const uint64_t want = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(w0) << 32) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(w2);
    const uint64_t got = eidx_hash(t ? w0 : 0u, t ? w1 : 0u, t ? w2 : 0u, t);
    if ((head & EIDX_VALID) && ((head >> 16) & 0xff) == nthr && wuni((uint32_t)(got == want))) {
      // published by an earlier decode of this sample: every lane starts
      // from its exact state (no sync rounds, no block scan)
      STAMP(3);
      STAMP(4);
      STAMP(5);
      if (a.dbg && t == 0) a.dbg[(uint64_t)k * 16 + 12] = ~0ull;  // index hit: no sync rounds
      zero_window_coefs(S, coef, t);
      if (active) {
        DecState g;
        g.pos = t ? w0 : 0u;
        g.z = t ? (int)(w1 & 0xff) : 0;
        g.ph = t ? (int)((w1 >> 8) & 0xff) : 0;
        const uint32_t cur = t ? w2 : 0u;
        start_blk = g.z == 0 ? cur : cur + 1;
        uint32_t it_lane2 = 0;
        if (g.pos < my_end)
          write_range(S, T, words, wuni(S.ds_bytes), g, my_end, cur, wave_uniform((gshort_t *)coef),
                      wuni(S.cf_bytes), wave_uniform((gshort_t *)dcd), wuni(S.dc_bytes), it_lane2, dc_diffs, rs0,
                      rs1, rs2);
      } else {
        start_blk = (uint32_t)S.nblocks;
      }
      publish_dc();
      return false;
    }
  }
  // ------------------------------------------------------------- P3 ----
  STAMP(3);
  DecState g;
  g.pos = active ? t * cbits : 0;
  g.z = 0;
  g.ph = 0;
  uint32_t my_cnt = 0;
  int my_nev = 0, my_cb = 0, my_eb = 0;  // events: count, buffer, block count of slot 0
  DecState e = g;
  uint32_t it_lane = 0, it_wave = 0;  // diagnostics: loop iterations (max over lanes per round)
  // event stride: NEV events spread over a lane's expected block count
  const uint32_t evq = ((uint32_t)S.nblocks / nthr + NEV) / NEV;
  const int esh = evq <= 1 ? 0 : 32 - __clz((int)(evq - 1));
  if (active) e = sync_range<false>(S, T, words, g, my_end, t, my_cnt, my_nev, my_cb, my_eb, g, esh, it_lane);
  if (a.dbg) it_wave += __reduce_max_sync(~0ull, it_lane);
  int rounds = 0;
  for (;;) {
    DecState ng;
    ng.pos = seg_prev(e.pos, t);
    ng.z = (int)seg_prev((uint32_t)e.z, t);
    ng.ph = (int)seg_prev((uint32_t)e.ph, t);
    const bool changed = active && t > 0 && (ng.pos != g.pos || ng.z != g.z || ng.ph != g.ph);
    if (!__any(changed)) break;
    rounds++;
    if (changed) {
      g = ng;
      if (g.pos >= my_end) {
        e = g;
        my_cnt = 0;
        my_nev = 0;
        my_eb = 0;
      } else {
        it_lane = 0;
        e = sync_range<true>(S, T, words, g, my_end, t, my_cnt, my_nev, my_cb, my_eb, e, esh, it_lane);
      }
    }
    if (a.dbg) it_wave += __reduce_max_sync(~0ull, changed ? it_lane : 0u);
  }
  if (!active) my_cnt = 0;
  if (a.dbg && t == 0) {
    a.dbg[(uint64_t)k * 16 + 12] = (uint64_t)rounds;
    a.dbg[(uint64_t)k * 16 + 13] = (uint64_t)nthr;
    a.dbg[(uint64_t)k * 16 + 14] = (uint64_t)it_wave;
  }

  // ------------------------------------------------------------- P4 ----
  STAMP(4);
  const uint32_t blk_base = seg_exscan(my_cnt);
  bool bad_lane = false;
  if (active) {
    int64_t cur = g.z == 0 ? (int64_t)blk_base : (int64_t)blk_base - 1;
    bad_lane = cur < 0 || (cur % S.bpm) != g.ph;  // inconsistent stream
  }
  const bool any_bad = seg_any(bad_lane, sg);
  if (rec && !any_bad) {  // publish this sample's converged lane states
    const int64_t cur = g.z == 0 ? (int64_t)blk_base : (int64_t)blk_base - 1;
    uint32_t w0 = active ? g.pos : 0u, w1 = active ? (uint32_t)g.z | ((uint32_t)g.ph << 8) : 0u,
             w2 = active ? (uint32_t)cur : 0u;
    const uint64_t h = eidx_hash(t ? w0 : 0u, t ? w1 : 0u, t ? w2 : 0u, t);
    if (t == 0) {  // lane 0's state is (0, 0, 0): its words carry the header and hash
      w0 = (uint32_t)(h >> 32);
      w1 = EIDX_VALID | (nthr << 16);
      w2 = (uint32_t)h;
    }
    rec[EIDX_WORDS * t] = w0;
    rec[EIDX_WORDS * t + 1] = w1;
    rec[EIDX_WORDS * t + 2] = w2;
  }

  // ------------------------------------------------------------- P5 ----
  STAMP(5);
  K1_STOP_AT(4, nthr != 0x7fffffffu, any_bad);  // diagnostics: K1 up to the sync pass (no write pass)
  zero_window_coefs(S, coef, t);
  uint32_t it_lane2 = 0;
  start_blk = blk_base;
  if (active && g.pos < my_end) {
    int64_t cur = g.z == 0 ? (int64_t)blk_base : (int64_t)blk_base - 1;
    if (cur >= 0)
      write_range(S, T, words, wuni(S.ds_bytes), g, my_end, (uint32_t)cur, wave_uniform((gshort_t *)coef),
                  wuni(S.cf_bytes), wave_uniform((gshort_t *)dcd), wuni(S.dc_bytes), it_lane2, dc_diffs, rs0, rs1,
                  rs2);
  }
  publish_dc();
  if (a.dbg) {
    const uint32_t wmax = __reduce_max_sync(~0ull, it_lane2);
    if (t == 0) a.dbg[(uint64_t)k * 16 + 15] = (uint64_t)wmax;
  }

  return any_bad;
}

// Bump-allocate this image's regions of the launch arena (wave-uniform; lane
// 0 does the atomic) and zero its window coefficients (the write pass stores
// only non-zero coefficients).  Region sizes: de-stuffed stream + padding,
// window coefficients (int16 x 64 per block), DC differences (int16 per
// block, coefficient output only), window planes (64 B per block), K2 band
// staging (crop RGB).
FFCV_DEV uint64_t align256(uint64_t x) { return (x + 255) & ~(uint64_t)255; }
FFCV_DEV int alloc_scratch(JShared &S, const JpegArgs &a, uint32_t nbytes, int t, int MODE, int k) {
  const uint64_t ds = align256((uint64_t)nbytes + 64), cf = align256((uint64_t)S.nwin * 128);
  // DC differences are stored only for the coefficient output (the other
  // modes predict DC from the write pass's per-lane running sums)
  const uint64_t dc = MODE == JM_COEF ? align256((uint64_t)S.nblocks * 2) : 0, pl = align256((uint64_t)S.nwin * 64);
  const uint64_t rgb = MODE == JM_RRC ? align256((uint64_t)S.rh * S.rw * 3) : 0;
  const uint64_t need = ds + cf + dc + pl + rgb;
  // An image larger than the whole arena reserves nothing (a 2400x1800 image
  // decoded first, largest-first, would otherwise hold the arena whenever its
  // give-back below loses the race, failing every image of the launch).  A
  // check against the live counter measured -1.5% (one more memory round
  // trip before the workgroup barrier).
  if (need > a.arena_bytes) {
    if (t == 0) a.info[k].arena_need = 0;
    return FFCV_SAMPLE_TOO_LARGE;
  }
  unsigned long long base = 0;
  if (t == 0) base = atomicAdd(a.arena_top, (unsigned long long)need);
  // readfirstlane returns int: widen through uint32_t (an offset at or past
  // 2^31 would otherwise sign-extend and read as TOO_LARGE)
  base = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
  if (base + need > a.arena_bytes) {
    // Arena exhausted.  Give the space back only if no reservation was made
    // after this one (the counter still ends at this image's region): a
    // compare-and-swap from base + need to base.  A plain subtract (round 3)
    // lowered the counter below a later image's live region whenever two
    // failures interleaved with a success, and the next image was handed
    // overlapping scratch.  When the swap fails the region stays reserved
    // (unused): the counter never goes below a live region.
    if (t == 0) {
      atomicCAS(a.arena_top, (unsigned long long)(base + need), (unsigned long long)base);
      a.info[k].arena_need = 0;
    }
    return FFCV_SAMPLE_TOO_LARGE;
  }
  if (t == 0) {
    a.info[k].arena_base = base;
    a.info[k].arena_need = need;
  }
  S.ds_off = base;
  S.ds_bytes = (uint32_t)ds;
  S.cf_off = base + ds;
  S.cf_bytes = (uint32_t)cf;
  S.dc_off = S.cf_off + cf;
  S.dc_bytes = (uint32_t)dc;
  const uint64_t pl_off = S.dc_off + dc;
  S.rgb_off = pl_off + pl;
  uint64_t o = pl_off;
  for (int c = 0; c < S.ncomp; c++) {
    const uint64_t wstride = (uint64_t)(S.wx1[c] - S.wx0[c] + 1) * 8;
    S.poff[c] = o - ((uint64_t)S.wy0[c] * 8 * wstride + (uint64_t)S.wx0[c] * 8);  // wraps: see ImgInfo
    o += wstride * (uint64_t)(S.wy1[c] - S.wy0[c] + 1) * 8;
  }
  return FFCV_SAMPLE_OK;
}

// K1 workgroup order: a workgroup's waves decode JW images and its LDS is
// held until the slowest one is done, so images of similar stream length
// (the best predictor of an image's K1 time) are grouped together: a
// one-workgroup counting sort of the batch by compressed size in 1 KB
// buckets, largest first, so the launch's last workgroups (its tail, which
// K1b and K2 wait for) hold its smallest images.  Only which wave decodes
// which image changes: every image is decoded the same way, and its outputs
// stay at its own index.
#define K1O_NB 128
#define K1O_T 1024
#define K1O_PER 16  // images per thread held in registers: launches up to 16,384 images in one pass
__global__ void __launch_bounds__(K1O_T) k1_order_kernel(JpegArgs a, uint32_t *order) {
  __shared__ uint32_t cnt[K1O_NB];
  const int t = threadIdx.x;
  if (t < K1O_NB) cnt[t] = 0;
  auto bucket_of = [](uint64_t size) -> int {
#ifdef K1O_ASCENDING
    return (int)min<uint64_t>(size >> 10, K1O_NB - 1);
#else
    return K1O_NB - 1 - (int)min<uint64_t>(size >> 10, K1O_NB - 1);
#endif
  };
  auto size_of = [&](int k) -> uint64_t {
    if (a.table) {
      const uint64_t id = a.ids[k];
      return id < a.n_table ? a.table[id].size : 0;
    }
    return a.samples[k].size;
  };
  // (round 4) every image's sample id, then its size, loaded with all of a
  // thread's images in flight, the buckets kept in registers for both passes:
  // the round-3 loop issued two dependent loads per image per pass in series
  // (~50-70 us per 12,288-image launch, ahead of every K1)
  uint64_t ids[K1O_PER];
#pragma unroll
  for (int i = 0; i < K1O_PER; i++) {
    const int k = t + i * K1O_T;
    ids[i] = a.table && k < a.batch ? a.ids[k] : 0;
  }
  int bk[K1O_PER];
#pragma unroll
  for (int i = 0; i < K1O_PER; i++) {
    const int k = t + i * K1O_T;
    uint64_t size = 0;
    if (k < a.batch) size = a.table ? (ids[i] < a.n_table ? a.table[ids[i]].size : 0) : a.samples[k].size;
    bk[i] = bucket_of(size);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < K1O_PER; i++)
    if (t + i * K1O_T < a.batch) atomicAdd(&cnt[bk[i]], 1u);
  for (int k = t + K1O_PER * K1O_T; k < a.batch; k += K1O_T) atomicAdd(&cnt[bucket_of(size_of(k))], 1u);
  __syncthreads();
  if (t < 64) {  // exclusive scan of the 128 bucket counts: one wave, two counts per lane
    const uint32_t c0 = cnt[2 * t], c1 = cnt[2 * t + 1];
    uint32_t x = c0 + c1;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (t >= d) x += y;
    }
    const uint32_t ex = x - c0 - c1;
    cnt[2 * t] = ex;
    cnt[2 * t + 1] = ex + c0;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < K1O_PER; i++) {
    const int k = t + i * K1O_T;
    if (k < a.batch) order[atomicAdd(&cnt[bk[i]], 1u)] = (uint32_t)k;
  }
  for (int k = t + K1O_PER * K1O_T; k < a.batch; k += K1O_T) order[atomicAdd(&cnt[bucket_of(size_of(k))], 1u)] = (uint32_t)k;
}

template <int MODE>
// Waves per SIMD K1 is compiled for: 4 (= the LDS limit, 16 images per CU)
// caps it at 128 VGPRs (a few spill, outside the decode loops); measured
// 1-2% faster than 3 (143 VGPRs) in the full pipeline.
#ifndef K1_WPE
#define K1_WPE 4
#endif
__global__ void __launch_bounds__(JW * JT) __attribute__((amdgpu_waves_per_eu(K1_WPE))) jpeg_entropy_kernel(JpegArgs a) {
  __shared__ K1Shared KS;
  const int wi = threadIdx.x / JL;  // image within the workgroup
  const int t = threadIdx.x % JL;   // lane within the image's segment
  const int sg = (threadIdx.x % JT) / JL;  // segment within the wave
  const int slot = blockIdx.x * (JW * IPW) + wi;
  const int k = a.k1_order && slot < a.batch ? (int)wuni(a.k1_order[slot]) : slot;
  JShared &S = KS.w[wi];
  const bool have = k < a.batch;
  ffcv_sample smp = {};
  int rng_err = 0;
  // The workgroup's draws (draw_kernel fused): all in wave 0, lane 3 w + part
  // for image w, so the MT19937 seeding chain runs once per workgroup instead
  // of once per wave; the crops are read by every wave's parse after the
  // barrier that follows the header staging (a workgroup fence: same CU)
  __shared__ int s_rngerr[JW * IPW];
  if (a.table && a.do_draw) {
    if (threadIdx.x < JT) {
      int err = 0;
      if (threadIdx.x < 3 * JW * IPW) {
        const int w = threadIdx.x / 3, part = threadIdx.x % 3;
        const int sw = blockIdx.x * (JW * IPW) + w;
        const int kw = a.k1_order && sw < a.batch ? (int)a.k1_order[sw] : sw;
        if (kw < a.batch) {
          const uint64_t idw = a.ids[kw];
          const uint32_t hw = idw < a.n_table ? a.table[idw].height : 1u, ww = idw < a.n_table ? a.table[idw].width : 1u;
          err = draw_part(part, kw, idw, hw, ww, a.dp, a.crops_w, a.cut_w, a.flips_w);
        }
      }
      const uint64_t eb = __ballot(err != 0);
      if (threadIdx.x < JW * IPW) s_rngerr[threadIdx.x] = ((eb >> (3 * threadIdx.x)) & 7ull) != 0;
    }
  }
  if (have) {
    if (a.table) {  // fused gather (gather_samples_kernel)
      const uint64_t id = a.ids[k];
      if (id < a.n_table) {
        smp = a.table[id];
      } else {  // out-of-range index: an empty jpg sample -> BAD_MARKER status
        smp.height = smp.width = 1;
      }
      if (t == 0 && a.samples_out) a.samples_out[k] = smp;
    } else {
      smp = a.samples[k];
    }
  }
  ImgInfo *info = a.info + k;
  const bool live = have && smp.mode == 0;
  if (have && smp.mode != 0 && t == 0) {  // raw samples are handled by rrc_raw_kernel / gather
    a.status[k] = FFCV_SAMPLE_OK;
    info->status = -1;  // K2 skips
  }
#ifdef K1_STOP
  if (have && t == 0) info->status = -1;  // diagnostics: K1b / K2 skip (K1 stops before writing the record)
#endif
  // no reservation until alloc_scratch makes one: an image that fails before
  // it (draws, parse, raw) must not report the previous launch's region
  // (ffcv_jpeg_arena_regions)
  if (have && t == 0) info->arena_need = 0;
  const uint8_t *src = wave_uniform(a.base + smp.offset);
  const uint32_t nbytes = wuni((uint32_t)smp.size);  // uniform: sizes buffer resources
  auto fail = [&]() {
    if (t == 0) {
      a.status[k] = S.status;
      info->status = S.status;
    }
    if (MODE == JM_FULL) {  // zero-fill (K2 does it for RRC)
      uint64_t bytes = (uint64_t)smp.height * smp.width * 3;
      uint8_t *o = (uint8_t *)a.out + a.out_stride * k;
      for (uint64_t i = t; i < bytes && i < a.out_stride; i += JL) o[i] = 0;
    }
  };

  // ------------------------------------------------------------- P0 ----
  STAMP(0);
  if (live) {
    // aligned dword loads (one batch per lane), bytes scattered into LDS
    const uint32_t nh = min(nbytes, (uint32_t)HDR_BYTES);
    const uint32_t mis = (uint32_t)((uintptr_t)src & 3);
    const uint32_t *aw = (const uint32_t *)(src - mis);
    constexpr int NW = (HDR_BYTES + 4) / 4;
#pragma unroll
    for (int r = 0; r < (NW + JL - 1) / JL; r++) {
      const int i = r * JL + t;
      const int b0 = 4 * i - (int)mis;
      const uint32_t w = i < NW && b0 < (int)nh ? gld_u32(aw + i) : 0u;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int idx = b0 + j;
        if (idx >= 0 && idx < HDR_BYTES) S.hdr[idx] = idx < (int)nh ? (uint8_t)(w >> (8 * j)) : 0;
      }
    }
  }
  if (a.table && a.do_draw) {  // the draws (wave 0) are done; waves 1.. staged their headers meanwhile
    __syncthreads();
    rng_err = s_rngerr[wi];
  } else {
    wsync_lds();
  }
  STAMP(10);
  K1_STOP_AT(7, smp.size != 0x7fffffffffffull);  // diagnostics: gather, draws and header staging
  if (t == 0) S.src = src;
  if (JL == JT || t == 0) {  // the whole wave runs the (scalar) parse; see parse_header
    int st = live ? (rng_err ? FFCV_SAMPLE_RNG : parse_header(S, wave_uniform(src), nbytes, smp, a, k, MODE)) : -1;
    if (st == FFCV_SAMPLE_OK) st = alloc_scratch(S, a, nbytes, t, MODE, k);
    if (t == 0) S.status = st;
  }
  __syncthreads();

  K1_STOP_AT(8, smp.size != 0x7fffffffffffull);  // diagnostics: up to the parse and the scratch allocation
  // ------------------------------------------------------------- P1 ----
  // The workgroup's first valid image provides the shared tables; every
  // image whose table slots and DHT bytes equal that image's uses them.
  STAMP(1);
  int ref = -1;
#pragma unroll
  for (int w = JW * IPW - 1; w >= 0; w--)
    if (KS.w[w].status == FFCV_SAMPLE_OK) ref = w;
  bool match = false;
  if (ref >= 0 && S.status == FFCV_SAMPLE_OK) {
    const JShared &R = KS.w[ref];
    const uint8_t *rsrc = R.src;
    match = R.nslots == S.nslots;
    for (int q = 0; q < NSLOT; q++)
      if (q < R.nslots && R.slot_tab[q] != S.slot_tab[q]) match = false;
    if (match && ref != wi) {
      bool diff = false;
      for (int q = 0; q < R.nslots; q++) {
        const uint32_t dr = R.dht_off[R.slot_tab[q]], ds = S.dht_off[S.slot_tab[q]];
        auto hb = [](const JShared &X, const uint8_t *xs, uint32_t p) -> int {
          return p < HDR_BYTES ? X.hdr[p] : gld_u8(xs + p);
        };
        int total = 0;
        for (int l = 0; l < 16; l++) total += hb(S, src, ds + l);
        for (int i = t; i < 16 + total; i += JL) diff |= hb(S, src, ds + i) != hb(R, rsrc, dr + i);
      }
      match = !seg_any(diff, sg);
    }
  }
  if (ref >= 0) {
    const JShared &R = KS.w[ref];
    const uint8_t *rsrc = R.src;
    auto HBR = [&](uint32_t p) -> int { return p < HDR_BYTES ? (int)R.hdr[p] : (int)gld_u8(rsrc + p); };
    build_tables<JW * JT>(KS.tab, R, HBR, (int)threadIdx.x);
  }
  // (no workgroup barrier below this point: each wave runs on its own)
  if (!live) return;
  if (S.status != FFCV_SAMPLE_OK) {
    fail();
    return;
  }
  auto HB = [&](uint32_t p) -> int {
    int v;
    if (p < HDR_BYTES)
      v = S.hdr[p];
    else
      v = gld_u8(src + p);
    return v;
  };
  JTables *gt = (JTables *)(a.gtab + a.gtab_slot * k);
  if (!match) build_tables<JL>(*gt, S, HB, t);
  if (t < 3) S.qmax[t] = 0;
  wsync_lds();
  for (int i = t; i < S.ncomp * 64; i += JL) {
    int c = i >> 6, zz = i & 63;
    int tq = S.tq[c];
    uint32_t q = S.dqt_off[tq];
    int qv = S.dqt_prec[tq] ? ((HB(q + 2 * zz) << 8) | HB(q + 2 * zz + 1)) : HB(q + zz);
    int n = c_natural[zz];
    const int16_t qmv = (int16_t)(((int64_t)qv * c_aanscales[n] + (1 << 11)) >> 12);
    info->qmul[c][n] = qmv;  // read by jpeg_idct_kernel only
    if (n != 0) atomicMax(&S.qmax[c], qmv < 0 ? -(int)qmv : (int)qmv);
  }
  wsync_lds();  // header bytes are dead from here (P2 stages into the same LDS)
  if (match ? KS.tab.bad : gt->bad) {
    if (t == 0) S.status = FFCV_SAMPLE_BAD_MARKER;
    wsync_lds();
    fail();
    return;
  }
  // the window coefficients were zeroed by alloc_scratch
  // arena offsets are wave-uniform: keep them in scalar registers
  const uint64_t cf_off = ((uint64_t)wuni((uint32_t)(S.cf_off >> 32)) << 32) | wuni((uint32_t)S.cf_off);
  int16_t *coef = (int16_t *)(a.arena + cf_off);

  K1_STOP_AT(1, cf_off != 0x7fffffffffffull);  // diagnostics: K1 up to the tables (no de-stuff)
  // ------------------------------------------------------------- P2 ----
  // De-stuffing in stream order: each step the wave reads 64 consecutive
  // aligned dwords of the segment (one per lane), keeps every byte except a
  // 0x00 after 0xFF, stops at the first marker (0xFF + non-zero), and
  // writes the kept bytes at offsets from a wave scan of their counts.
  STAMP(2);
  uint8_t *gds = a.arena + (((uint64_t)wuni((uint32_t)(S.ds_off >> 32)) << 32) | wuni((uint32_t)S.ds_off));
  uint32_t dlen = 0;
  {
    const uint32_t seg0 = wuni(S.scan_off);  // uniform: sizes the buffer resource below
    const uint32_t seglen = nbytes > seg0 ? nbytes - seg0 : 0;
    const uintptr_t sb = (uintptr_t)(src + seg0);
    const uint32_t mis = (uint32_t)(sb & 3);
    const uint32_t *aw = (const uint32_t *)(sb - mis);
    const uint32_t ndw = (seglen + mis + 3) / 4;
    uint32_t carry = 0;  // byte before this step's first byte (0: none / not 0xFF)
    // Kept bytes are staged in LDS and flushed to HBM as aligned dwords every
    // DS_FLUSH steps: a byte store per kept byte would make every prefetch
    // wait behind the stores (gfx9 counts loads and stores in one vmcnt).
    uint32_t fbase = 0;  // stream offset of stage[0] (a multiple of 4)
    // The flush issues a fixed number of buffer stores per lane (out of range
    // past the staged bytes), so the prefetched loads issued before it are
    // waited for with a static vmcnt, not behind a dynamic store count.
    const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(wave_uniform(gds), 0, (int)wuni(S.ds_bytes), BUF_CFG);
    constexpr int FL_N = (STAGE_BYTES / 4 + JL - 1) / JL;  // stores per lane per flush
    auto flush = [&](uint32_t upto) {  // write stage bytes [fbase, upto), upto % 4 == 0
      wsync_lds();
      const uint32_t nd = (upto - fbase) / 4;
#pragma unroll
      for (int f = 0; f < FL_N; f++) {
        const uint32_t q = (uint32_t)(f * JL + t);
        const uint32_t v = ((const uint32_t *)S.stage)[min(q, (uint32_t)(STAGE_BYTES / 4 - 1))];
        __builtin_amdgcn_raw_buffer_store_b32(v, drs, q < nd ? fbase + 4 * q : BUF_OOR, 0, 0);
      }
      wsync_lds();
    };
    // DS_DEPTH-deep prefetch ring, unrolled so every ring register is consumed in
    // place (a rotating copy would make the compiler wait for all loads)
    // segment dwords through a buffer resource: past the segment the load is
    // out of range and returns 0 with no access, so every step issues its
    // load unconditionally and the compiler can count vmcnt statically
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc((void *)wave_uniform(aw), 0, (int)(ndw * 4), BUF_CFG);
    auto ld = [&](uint32_t d) -> uint32_t { return __builtin_amdgcn_raw_buffer_load_b32(srs, d * 4, 0, 0); };
    // Each lane takes two consecutive dwords per step (8 bytes): the step's
    // fixed work -- the wave scan of the kept counts, the neighbour bytes,
    // the marker ballot, the ring bookkeeping -- is shared by twice the bytes.
    // Byte masks stay in 0x80-per-byte form (zm), so no multiply gathers bits.
    constexpr int D2 = DS_DEPTH / 2;  // ring depth in two-dword lane steps
    static_assert(DS_FLUSH == DS_DEPTH, "one flush per ring cycle");
    uint32_t r0[D2], r1[D2];
#pragma unroll
    for (int u = 0; u < D2; u++) {
      r0[u] = ld(2 * (u * JL + t));
      r1[u] = ld(2 * (u * JL + t) + 1);
    }
    bool done = false;
    auto zm = [](uint32_t x) { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u; };
    // kept / marker bytes of one dword (0x80 per byte) at stream index rel0 of its byte 0
    auto scan_dw = [&](uint32_t w, uint32_t prevb, uint32_t nextb, int rel0, uint32_t &keep, uint32_t &mark) {
      const uint32_t pw = (w << 8) | prevb;          // previous byte of each byte
      const uint32_t nw = (w >> 8) | (nextb << 24);  // next byte of each byte
      const int lo = max(0, -rel0), hi = min(4, (int)seglen - rel0);  // valid bytes [lo, hi)
      const uint32_t vhi = hi >= 4 ? 0x80808080u : (hi <= 0 ? 0u : 0x80808080u >> (32 - 8 * hi));
      const uint32_t valid = vhi & (0x80808080u << (8 * lo));
      const uint32_t ff = zm(~w);
      // a 0x00 after 0xFF is stuffing, except the segment's first byte
      const uint32_t head = rel0 <= 0 ? 0x80808080u >> (24 - 8 * min(3, -rel0)) : 0u;  // bytes with rel <= 0
      const uint32_t removed = zm(w) & zm(~pw) & ~head;
      // a marker is 0xFF followed by a non-zero byte; end of data acts as one
      const uint32_t lastm = (hi >= 1 && rel0 + hi == (int)seglen) ? 0x80u << (8 * (hi - 1)) : 0u;
      mark = ((ff & ~zm(nw)) | (ff & lastm)) & valid;
      keep = valid & ~removed;
    };
    for (uint32_t base2 = 0; !done; base2 += D2 * JL) {
#pragma unroll
      for (int u = 0; u < D2; u++) {
        const uint32_t base = base2 + u * JL;  // two-dword lane step of lane 0
        const uint32_t w0 = r0[u], w1 = r1[u];
        const uint32_t nd = 2 * (base + D2 * JL + t);
        r0[u] = ld(nd);  // issued on every step (see srs)
        r1[u] = ld(nd + 1);
        if (done || 2 * base >= ndw) {
          done = true;
          continue;
        }
        const uint32_t d0 = 2 * (base + t);
        const uint32_t w1prev = lane_prev(w1);
        const uint32_t w0next = lane_next(w0);
        const uint32_t nfirst = seg_read(r0[(u + 1) % D2], 0, sg);  // next step's first dword
        const uint32_t prevb = t == 0 ? carry : (w1prev >> 24);
        const uint32_t next1 = (t == JL - 1 ? nfirst : w0next) & 0xff;
        const int rel0 = (int)(4 * d0) - (int)mis;  // stream index of w0's byte 0
        uint32_t k0, m0, k1, m1;
        scan_dw(w0, prevb, w1 & 0xff, rel0, k0, m0);
        scan_dw(w1, w0 >> 24, next1, rel0 + 4, k1, m1);
        // the first marker of the step ends the segment: keep the bytes before it
        const uint32_t b0 = m0 ? (m0 & (0u - m0)) - 1u : 0xffffffffu;
        const uint32_t b1 = m0 ? 0u : (m1 ? (m1 & (0u - m1)) - 1u : 0xffffffffu);
        k0 &= b0;
        k1 &= b1;
        const uint64_t mk = seg_ballot((m0 | m1) != 0, sg);
        if (mk) {
          const int ml = __ffsll((unsigned long long)mk) - 1;
          if (t > ml) k0 = k1 = 0;
          done = true;
        }
        const uint32_t c0 = __popc(k0), cnt = c0 + __popc(k1);
        const uint32_t off = dlen + seg_exscan(cnt) - fbase;
#pragma unroll
        for (int j = 0; j < 8; j++) {  // branch-free: dropped bytes go to a dummy byte
          const uint32_t km = j < 4 ? k0 : k1, w = j < 4 ? w0 : w1;
          const int jj = j & 3;
          const bool kj = (km >> (8 * jj + 7)) & 1;
          const uint32_t before = (j < 4 ? 0u : c0) + (jj ? __popc(km & ((1u << (8 * jj)) - 1u)) : 0u);
          S.stage[kj ? off + before : STAGE_DUMMY] = (uint8_t)(w >> (8 * jj));
        }
        dlen = seg_read(off + cnt, JL - 1, sg) + fbase;
        carry = seg_read(w1, JL - 1, sg) >> 24;
      }
      if (!done) {  // flush whole dwords, keep the 0..3-byte tail
        const uint32_t upto = dlen & ~3u;
        flush(upto);
        if (t < (int)(dlen - upto)) S.stage[t] = S.stage[upto - fbase + t];
        fbase = upto;
        wsync_lds();
      }
    }
    // tail + zero padding (libjpeg fills zeros after a marker)
    wsync_lds();
    for (uint32_t i = dlen - fbase + t; i < dlen - fbase + STREAM_PAD + 4; i += JL) S.stage[i] = 0;
    flush((dlen + STREAM_PAD + 3) & ~3u);
  }
  wsync_mem();
  K1_STOP_AT(2, dlen != 0x7fffffffu);  // diagnostics: K1 up to the de-stuffed stream
  // one image per wave: its stream base is wave-uniform (scalar registers,
  // so the refill loads use the scalar-base + 32-bit offset form)
  const uint32_t *words = wave_uniform((const uint32_t *)gds);
  const uint32_t total_bits = dlen * 8;


  int16_t *dcd = (int16_t *)(a.arena + (((uint64_t)wuni((uint32_t)(S.dc_off >> 32)) << 32) | wuni((uint32_t)S.dc_off)));
  const uint64_t sid = a.ids && a.eidx ? a.ids[k] : ~0ull;
  const bool any_bad = match ? entropy_passes(S, KS.tab, a, k, t, sg, words, total_bits, coef, dcd, sid, MODE == JM_COEF)
                             : entropy_passes(S, *gt, a, k, t, sg, words, total_bits, coef, dcd, sid, MODE == JM_COEF);
  wsync_mem();
  K1_STOP_AT(5, !any_bad);  // diagnostics: K1 up to the write pass

  // ------------------------------------------------------------- P6 ----
  // DC prediction (jdhuff.c last_dc_val) for the coefficient output (JM_COEF;
  // the other modes run it in jpeg_idct_kernel): per-component running sum of
  // DC differences in MCU block order, as a wave scan over block ranges of a
  // multiple of 8 blocks read as 16-byte buffer loads, DCP_U in flight.
  STAMP(6);
  if (MODE == JM_COEF) {
    constexpr int DCP_U = 4;
    const int nb = S.nblocks, bpm = S.bpm;
    const int per_b = ((nb + JL - 1) / JL + 7) & ~7;
    const int b0 = min(nb, per_b * t), b1 = min(nb, per_b * (t + 1));
    const __amdgpu_buffer_rsrc_t drs =
        __builtin_amdgcn_make_buffer_rsrc(wave_uniform((void *)dcd), 0, (int)wuni(S.dc_bytes), BUF_CFG);
    auto load8 = [&](int q) -> uint4 {  // blocks b0 + 8q .. b0 + 8q + 7
      const int b = b0 + 8 * q;
      return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                           drs, b < b1 ? (uint32_t)b * 2 : BUF_OOR, 0, 0));
    };
    auto diff = [](const uint4 &w, int e) -> int {
      const uint32_t x = e < 2 ? w.x : e < 4 ? w.y : e < 6 ? w.z : w.w;
      return (int)(int16_t)(x >> (16 * (e & 1)));
    };
    int32_t s0 = 0, s1 = 0, s2 = 0;  // (registers: no dynamically indexed arrays)
    int ph = b0 % bpm;
    for (int q0 = 0; q0 * 8 < per_b; q0 += DCP_U) {
      uint4 w[DCP_U];
#pragma unroll
      for (int u = 0; u < DCP_U; u++) w[u] = load8(q0 + u);
#pragma unroll
      for (int u = 0; u < DCP_U; u++)
#pragma unroll
        for (int e = 0; e < 8; e++) {
          if (b0 + 8 * (q0 + u) + e < b1) {
            const int c = S.blk_comp[ph], d = diff(w[u], e);
            s0 += c == 0 ? d : 0;
            s1 += c == 1 ? d : 0;
            s2 += c == 2 ? d : 0;
            if (++ph == bpm) ph = 0;
          }
        }
    }
    int32_t p0 = seg_exscan_i(s0), p1 = seg_exscan_i(s1), p2 = seg_exscan_i(s2);
    ph = b0 % bpm;
    int m = b0 / bpm;
    int my = m / S.mcux, mx = m - my * S.mcux;
    for (int q0 = 0; q0 * 8 < per_b; q0 += DCP_U) {
      uint4 w[DCP_U];
#pragma unroll
      for (int u = 0; u < DCP_U; u++) w[u] = load8(q0 + u);
#pragma unroll
      for (int u = 0; u < DCP_U; u++)
#pragma unroll
        for (int e = 0; e < 8; e++) {
          if (b0 + 8 * (q0 + u) + e < b1) {
            const int c = S.blk_comp[ph], d = diff(w[u], e);
            p0 += c == 0 ? d : 0;
            p1 += c == 1 ? d : 0;
            p2 += c == 2 ? d : 0;
            const int pv = c == 0 ? p0 : (c == 1 ? p1 : p2);
            const int bx = mx * S.hs[c] + S.blk_dx[ph], by = my * S.vs[c] + S.blk_dy[ph];
            if (bx >= S.wx0[c] && bx <= S.wx1[c] && by >= S.wy0[c] && by <= S.wy1[c])
              coef[(S.coff[c] + (uint64_t)(by - S.wy0[c]) * (S.wx1[c] - S.wx0[c] + 1) + (bx - S.wx0[c])) * 64] =
                  (int16_t)pv;
            if (++ph == bpm) {
              ph = 0;
              if (++mx == S.mcux) {
                mx = 0;
                my++;
              }
            }
          }
        }
    }
  }
  wsync_mem();
  K1_STOP_AT(6, !any_bad);  // diagnostics: K1 up to the DC prediction

  if (MODE == JM_COEF) {
    int16_t *o = (int16_t *)a.out + a.out_stride / 2 * k;
    for (int64_t b = t; b < S.nblocks; b += JL) {
      int64_t m = b / S.bpm;
      int ph = (int)(b - m * S.bpm);
      int my = (int)(m / S.mcux), mx = (int)(m - (int64_t)my * S.mcux);
      int c = S.blk_comp[ph];
      int bx = mx * S.hs[c] + S.blk_dx[ph], by = my * S.vs[c] + S.blk_dy[ph];
      const int16_t *cp = coef + (S.coff[c] + (uint64_t)by * (S.wx1[c] - S.wx0[c] + 1) + bx) * 64;  // window = image
      int16_t zz[64], nb[64];
#pragma unroll
      for (int p8 = 0; p8 < 8; p8++) *(uint4 *)(zz + p8 * 8) = ((const uint4 *)cp)[p8];
#pragma unroll
      for (int n = 0; n < 64; n++) nb[n] = zz[kZigzagOfNatural[n]];
      uint4 *dp = (uint4 *)(o + b * 64);
#pragma unroll
      for (int p8 = 0; p8 < 8; p8++) dp[p8] = *(const uint4 *)(nb + p8 * 8);
    }
    if (t == 0) a.status[k] = any_bad ? FFCV_SAMPLE_CORRUPT : FFCV_SAMPLE_OK;
    return;
  }

  // ------------------------------------------------------------- P7 ----
  // geometry + crop window for K2
  STAMP(7);
  if (t == 0) {
    info->status = FFCV_SAMPLE_OK;
    info->W = S.W;
    info->H = S.H;
    info->ncomp = S.ncomp;
    info->color_rgb = S.color_rgb;
    for (int c = 0; c < 3; c++) {
      bool v = c < S.ncomp;
      info->he[c] = v ? S.hmax / S.hs[c] : 1;
      info->ve[c] = v ? S.vmax / S.vs[c] : 1;
      info->cw[c] = v ? S.cw[c] : 0;
      info->ch[c] = v ? S.ch[c] : 0;
      info->stride[c] = v ? (S.wx1[c] - S.wx0[c] + 1) * 8 : 0;
      info->poff[c] = v ? S.poff[c] : 0;
    }
    info->rgb_off = S.rgb_off;
    info->cf_off = S.cf_off;
    info->nblocks = S.nblocks;
    info->bpm = S.bpm;
    info->mcux = S.mcux;
    for (int c = 0; c < 3; c++) {
      info->coff[c] = S.coff[c];
      info->hs[c] = S.hs[c];
      info->vs[c] = S.vs[c];
      info->wx0[c] = S.wx0[c];
      info->wx1[c] = S.wx1[c];
      info->wy0[c] = S.wy0[c];
      info->wy1[c] = S.wy1[c];
      info->qmax[c] = S.qmax[c];
    }
    for (int b = 0; b < 10; b++) {
      info->blk_comp[b] = S.blk_comp[b];
      info->blk_dx[b] = S.blk_dx[b];
      info->blk_dy[b] = S.blk_dy[b];
    }
    info->ri = S.ri;
    info->rj = S.rj;
    info->rh = S.rh;
    info->rw = S.rw;
    a.status[k] = any_bad ? FFCV_SAMPLE_CORRUPT : FFCV_SAMPLE_OK;
  }
  if (MODE == JM_RRC) {  // the resize plan and linear taps K2's workgroups share
    const int out_h = a.p.out_h, out_w = a.p.out_w;
    const ResizePlan P = make_plan(S.rw, S.rh, out_w, out_h);
    const bool tabs = a.taps && P.kind == 3 && out_w + out_h <= K2_TAPS;
    if (tabs) {
      const int flip = a.flips ? a.flips[k] : 0;
      uint2 *tp = a.taps + (uint64_t)k * K2_TAPS;
      for (int i = t; i < out_w + out_h; i += JL)
        tp[i] = tap_pack(i < out_w ? lin_tap(P.scale_x, P.inv_x, P.sw, flip ? out_w - 1 - i : i)
                                   : lin_tap(P.scale_y, P.inv_y, P.sh, i - out_w));
    }
    if (t == 0) {
      info->plan = P;
      info->taps = tabs;
    }
  }

  // (P8, the DC prediction and the IDCT of the window's blocks, is
  // jpeg_idct_kernel: a launch of its own runs it at VALU throughput instead of
  // behind this kernel's latency-bound waves, ~25% of K1's time per image)
  STAMP(9);
}

// ======================================================================= //
// K1b: DC prediction + de-zigzag + dequantise + ifast IDCT (jidctfst.c)   //
// ======================================================================= //
// One 256-thread workgroup per image; every thread IDCTs window blocks
// i = t, t + 256, ... into the window planes K2 reads.  The DC prediction
// (jdhuff.c last_dc_val) is done by K1's write pass as running sums per lane:
// the absolute DC of a block is its slot 0 plus the offset of the lane that
// started it (a 6-step search over the lanes' start blocks).
constexpr int K1B_T = 256;

__global__ void __launch_bounds__(K1B_T) jpeg_idct_kernel(JpegArgs a) {
  __shared__ ImgInfo L;  // this image's record (per-thread component lookups read LDS)
  const int k = blockIdx.x, t = threadIdx.x;
  const ImgInfo &G = a.info[k];
  if (G.status != FFCV_SAMPLE_OK) return;  // failed (K2 zero-fills) or raw (-1)
  static_assert(sizeof(ImgInfo) % 4 == 0, "ImgInfo copies as dwords");
  for (int i = t; i < (int)(sizeof(ImgInfo) / 4); i += K1B_T) ((uint32_t *)&L)[i] = ((const uint32_t *)&G)[i];
  __syncthreads();
  int16_t *coef = (int16_t *)(a.arena + L.cf_off);
  uint8_t *planes = a.arena;
  int nbw[3];
#pragma unroll
  for (int c = 0; c < 3; c++) nbw[c] = c < L.ncomp ? (L.wx1[c] - L.wx0[c] + 1) * (L.wy1[c] - L.wy0[c] + 1) : 0;
  const int ntot = nbw[0] + nbw[1] + nbw[2];
  for (int i = t; i < ntot; i += K1B_T) {
    int c = 0, j = i;
    if (j >= nbw[0]) {
      j -= nbw[0];
      c = 1;
      if (j >= nbw[1]) {
        j -= nbw[1];
        c = 2;
      }
    }
    const int wbw = L.wx1[c] - L.wx0[c] + 1;
    const int by = L.wy0[c] + j / wbw, bx = L.wx0[c] + j % wbw;
    const int stride = wbw * 8;
    // block (c, bx, by) in MCU order, then the lane that started it: its
    // running DC sum in slot 0 plus that lane's offset is the absolute DC
    const int hs = L.hs[c], vs = L.vs[c];
    const int mx = bx / hs, my = by / vs, dx = bx - mx * hs, dy = by - my * vs;
    int ph = 0;
    for (int q = 0; q < L.bpm; q++)
      if (L.blk_comp[q] == c && L.blk_dx[q] == dx && L.blk_dy[q] == dy) ph = q;
    const uint32_t b = (uint32_t)((my * L.mcux + mx) * L.bpm + ph);
    int lane = 0;  // K1 wrote lane_blk0 / lane_off for its JL lanes only
#pragma unroll
    for (int st = JL / 2; st >= 1; st >>= 1)
      if (lane + st < JL && L.lane_blk0[lane + st] <= b) lane += st;
    idct_block(coef + (L.coff[c] + (uint64_t)j) * 64, L.qmul[c], L.qmax[c],
               planes + L.poff[c] + (uint64_t)by * 8 * stride + bx * 8, stride, L.lane_off[c][lane]);
  }
}

// ======================================================================= //
// K2: fancy upsampling + colour conversion into LDS, INTER_AREA + epilogue //
// ======================================================================= //

// Plane accessors: a component plane in HBM (GPlane) or a tile of it staged
// in LDS (TPlane, rows [r0, ..] x cols [c0, ..] of the plane).
struct GPlane {
  const uint8_t *p;
  int stride;
  FFCV_DEV int at(int r, int c) const { return p[(uint64_t)r * stride + c]; }
};
struct TPlane {
  const uint8_t *p;
  int r0, c0, pitch;
  FFCV_DEV int at(int r, int c) const { return p[__mul24(r - r0, pitch) + (c - c0)]; }  // tiles < 2^24 B
};

// jdsample.c upsampling of one component at full-resolution sample (y, x),
// with libjpeg's context-row edge replication.
template <class PL>
FFCV_DEV int upsample_at(const PL &P, int cw, int ch, int he, int ve, int y, int x) {
  auto clampr = [&](int r) { return r < 0 ? 0 : (r >= ch ? ch - 1 : r); };
  if (he == 1 && ve == 1) return P.at(y, x);
  if (he == 2 && ve == 1) {
    int col = x >> 1;
    if (cw <= 2) return P.at(y, col);
    int cur = P.at(y, col) * 3;
    if (x & 1) {
      if (col + 1 >= cw) return P.at(y, col);
      return (cur + P.at(y, col + 1) + 2) >> 2;
    }
    if (col == 0) return P.at(y, 0);
    return (cur + P.at(y, col - 1) + 1) >> 2;
  }
  if (he == 1 && ve == 2) {
    int r = y >> 1, other = (y & 1) ? r + 1 : r - 1;
    int sum = P.at(clampr(r), x) * 3 + P.at(clampr(other), x);
    return (sum + ((y & 1) ? 2 : 1)) >> 2;
  }
  if (he == 2 && ve == 2) {
    int r = y >> 1, col = x >> 1;
    if (cw <= 2) return P.at(r, col);
    int other = (y & 1) ? r + 1 : r - 1;
    int rc = clampr(r), oc = clampr(other);
    int thiss = P.at(rc, col) * 3 + P.at(oc, col);
    if (x & 1) {
      int nxt = col + 1 < cw ? P.at(rc, col + 1) * 3 + P.at(oc, col + 1) : thiss;
      return (thiss * 3 + nxt + 7) >> 4;
    }
    int last = col > 0 ? P.at(rc, col - 1) * 3 + P.at(oc, col - 1) : thiss;
    return (thiss * 3 + last + 8) >> 4;
  }
  return P.at(y / ve, x / he);  // int_upsample
}

// jdcolor.c ycc_rgb_convert with build_ycc_rgb_table's fixed point
FFCV_DEV void ycc_rgb(int y, int cb, int cr, int out[3]) {
  int x_cb = cb - 128, x_cr = cr - 128;
  out[0] = sat_u8i(y + ((91881 * x_cr + 32768) >> 16));
  out[1] = sat_u8i(y + ((-22554 * x_cb + 32768 + -46802 * x_cr) >> 16));
  out[2] = sat_u8i(y + ((116130 * x_cb + 32768) >> 16));
}

// The per-image fields the colour pass needs, held in registers.
struct ColorGeom {
  int ncomp, color_rgb;
  int he[3], ve[3], cw[3], ch[3];
};
// The part of an image record K2 reads (ImgInfo up to and including `taps`),
// fetched with ONE vector load per lane (lane i: dword i) at the top of the
// kernel together with the LUT, tap and epilogue loads, then broadcast to
// scalar registers with v_readlane.  Reading the fields from the global
// record where they are used issued them in ~6 dependent round trips (the
// compiler may not hoist loads above the status / mode branches), which was
// most of K2's per-workgroup fixed cost.
// Round 5: the head read through the scalar cache instead (s_load: no
// v_readlane per field, 49 VALU per wave; K2REC_SMEM=0 restores the vector
// load + broadcast for A/B runs).
#define K2REC_DW ((int)((offsetof(ImgInfo, taps) + 4) / 4))
static_assert(K2REC_DW <= 64, "record head fits one wave's lanes");
#ifndef K2REC_SMEM
#define K2REC_SMEM 1
#endif
struct K2Rec {
#if K2REC_SMEM
  const __attribute__((address_space(4))) uint32_t *p;  // the record (written by K1: a previous kernel)
  FFCV_DEV void load(const ImgInfo *rec, int) { p = (const __attribute__((address_space(4))) uint32_t *)rec; }
  FFCV_DEV uint32_t u(int i) const { return p[i]; }
#else
  uint32_t w;  // this lane's dword of the record head
  FFCV_DEV void load(const ImgInfo *rec, int t) { w = (t & 63) < K2REC_DW ? ((const uint32_t *)rec)[t & 63] : 0u; }
  FFCV_DEV uint32_t u(int i) const { return (uint32_t)__builtin_amdgcn_readlane((int)w, i); }
#endif
  FFCV_DEV int32_t s(int i) const { return (int32_t)u(i); }
  FFCV_DEV uint64_t u64(int i) const { return (uint64_t)u(i) | ((uint64_t)u(i + 1) << 32); }
  FFCV_DEV double f64(int i) const { return __builtin_bit_cast(double, u64(i)); }
};
#define K2F(f) ((int)(offsetof(ImgInfo, f) / 4))
FFCV_DEV ImgInfo k2_head(const K2Rec &R) {
  ImgInfo I;  // only the head fields are set (SROA keeps them in registers)
  I.status = R.s(K2F(status));
  I.W = R.s(K2F(W));
  I.H = R.s(K2F(H));
  I.ncomp = R.s(K2F(ncomp));
  I.color_rgb = R.s(K2F(color_rgb));
#pragma unroll
  for (int c = 0; c < 3; c++) {
    I.he[c] = R.s(K2F(he) + c);
    I.ve[c] = R.s(K2F(ve) + c);
    I.cw[c] = R.s(K2F(cw) + c);
    I.ch[c] = R.s(K2F(ch) + c);
    I.stride[c] = R.s(K2F(stride) + c);
    I.poff[c] = R.u64(K2F(poff) + 2 * c);
  }
  I.ri = R.s(K2F(ri));
  I.rj = R.s(K2F(rj));
  I.rh = R.s(K2F(rh));
  I.rw = R.s(K2F(rw));
  I.rgb_off = R.u64(K2F(rgb_off));
  I.plan.sw = R.s(K2F(plan.sw));
  I.plan.sh = R.s(K2F(plan.sh));
  I.plan.dw = R.s(K2F(plan.dw));
  I.plan.dh = R.s(K2F(plan.dh));
  I.plan.kind = R.s(K2F(plan.kind));
  I.plan.isx = R.s(K2F(plan.isx));
  I.plan.isy = R.s(K2F(plan.isy));
  I.plan.vec_end = R.s(K2F(plan.vec_end));
  I.plan.scale_x = R.f64(K2F(plan.scale_x));
  I.plan.scale_y = R.f64(K2F(plan.scale_y));
  I.plan.inv_x = R.f64(K2F(plan.inv_x));
  I.plan.inv_y = R.f64(K2F(plan.inv_y));
  I.taps = R.s(K2F(taps));
  return I;
}

FFCV_DEV ColorGeom color_geom(const ImgInfo &I) {
  ColorGeom g;
  g.ncomp = I.ncomp;
  g.color_rgb = I.color_rgb;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    g.he[c] = I.he[c];
    g.ve[c] = I.ve[c];
    g.cw[c] = I.cw[c];
    g.ch[c] = I.ch[c];
  }
  return g;
}

template <class PL>
FFCV_DEV void pixel_rgb(const ColorGeom &I, const PL *pl, int Y, int X, int v[3]) {
  if (I.ncomp == 1) {
    v[0] = v[1] = v[2] = pl[0].at(Y, X);
    return;
  }
  int s0 = upsample_at(pl[0], I.cw[0], I.ch[0], I.he[0], I.ve[0], Y, X);
  int s1 = upsample_at(pl[1], I.cw[1], I.ch[1], I.he[1], I.ve[1], Y, X);
  int s2 = upsample_at(pl[2], I.cw[2], I.ch[2], I.he[2], I.ve[2], Y, X);
  if (I.color_rgb) {
    v[0] = s0;
    v[1] = s1;
    v[2] = s2;
  } else {
    ycc_rgb(s0, s1, s2, v);
  }
}

// h2v2 fancy upsampling (jdsample.c h2v2_fancy_upsample) of the 2x2 output
// quad that chroma sample (R, C) expands to: q[0..3] = (2R,2C), (2R,2C+1),
// (2R+1,2C), (2R+1,2C+1).  Same arithmetic as upsample_at(he=ve=2, cw>2),
// with the 3x3 neighbourhood read once.
template <class PL>
FFCV_DEV void upsample_quad_h2v2(const PL &P, int cw, int ch, int R, int C, int q[4]) {
  const int ru = max(R - 1, 0), rd = min(R + 1, ch - 1);
  const int cl = max(C - 1, 0), cr = min(C + 1, cw - 1);
  const int ml = P.at(R, cl), mc = P.at(R, C), mr = P.at(R, cr);
  const int tl = 3 * ml + P.at(ru, cl), tc = 3 * mc + P.at(ru, C), tr = 3 * mr + P.at(ru, cr);
  const int bl = 3 * ml + P.at(rd, cl), bc = 3 * mc + P.at(rd, C), br = 3 * mr + P.at(rd, cr);
  const bool first = C == 0, last = C + 1 >= cw;
  q[0] = (3 * tc + (first ? tc : tl) + 8) >> 4;
  q[1] = (3 * tc + (last ? tc : tr) + 7) >> 4;
  q[2] = (3 * bc + (first ? bc : bl) + 8) >> 4;
  q[3] = (3 * bc + (last ? bc : br) + 7) >> 4;
}

struct LdsRoi {  // crop rows [row0, row0 + nrows), staged as RGB in LDS
  const uint8_t *p;
  int row0;
  int step;
  FFCV_DEV int at(int y, int x, int c) const { return p[__mul24(y - row0, step) + x * 3 + c]; }
  FFCV_DEV const uint8_t *pix(int y, int x) const { return p + __mul24(y - row0, step) + x * 3; }
};

// K2's FP16 LUT in LDS is channel-major, [c][256] halves (a.p.lut is [v][c]):
// entry (v, c) is v shifted plus the ds_read's immediate offset c * 512,
// where the interleaved v * 3 + c compiled to a 64-bit multiply-add per read
typedef __attribute__((address_space(3))) uint16_t lds_u16_t;
FFCV_DEV uint32_t lut_at(const lds_u16_t *L, int v, int c) { return L[(uint32_t)v + 256u * (uint32_t)c]; }
FFCV_DEV uint16_t lut_src(const uint16_t *lut, int d) { return lut[(d & 255) * 3 + (d >> 8)]; }  // LDS entry d
// The linear walk's last step, VResizeLinearVec's (m0 + m1 + 2) >> 2 of the
// vertical sum x = m0 + m1: the u8 value, or (FP16) the LDS byte address of
// its channel-0 LUT entry, base + 2 * ((x + 2) >> 2) = (x + lq) >> 1 & ~1 with
// lq = 2 + 2 * base (base even): an add3, a shift and an and, where indexing
// the value cost a 4-cycle shift-add more (tools/op_rate); lut_ld reads the
// channel-c entry at that address (channel c's table: + 512 c bytes)
template <bool FP16>
FFCV_DEV uint32_t lut_q(uint32_t x, uint32_t lq) { return FP16 ? ((x + lq) >> 1) & ~1u : (x + 2u) >> 2; }
FFCV_DEV uint32_t lut_base(const lds_u16_t *L) { return (uint32_t)(uintptr_t)L; }
FFCV_DEV uint32_t lut_ld(uint32_t q, int c) { return ((const lds_u16_t *)(uintptr_t)q)[256 * c]; }

#ifndef K2_WPE
#define K2_WPE 6  // waves per SIMD K2 is compiled for (6 WGs per CU at K2_LDS)
#endif
#ifndef K2_SADDR_STORE
#define K2_SADDR_STORE 1  // 0: the linear walk's per-row 64-bit output address (A/B builds)
#endif
#ifndef K2_AREA_FAST
#define K2_AREA_FAST 1  // 0: area crops take the general per-pixel path (A/B builds)
#endif

// K2's area walk: ResizeArea_Invoker (resize.cpp, INTER_AREA with both scales
// in [1, 2)) for output columns dx0, dx0 + 1 over this thread's row group, from
// the band's packed RGB rows in LDS (crop column x at byte xoff3 + 3 x of LDS
// row r - r0).  Same arithmetic and order as resize_area: per source row the
// horizontal sums buf = S[lo] a0 + S[lo + 1] a1 + S[lo + 2] a2 (a fixed
// 3-tap body: a destination index at a scale < 2 covers at most 3 source
// indices, and a tap past hi has weight 0, so x + S * 0 == x for these
// non-negative sums), then sum = beta(lo) buf(lo), sum += beta(r) buf(r).
// Consecutive output rows share at most their boundary source row, so one
// cached row of sums covers the reuse.  The two columns' values of a channel
// form one float2 (v_pk_mul_f32 / v_pk_add_f32: each lane is an ordinary
// IEEE multiply or add, contraction off).  A row group is two whole waves: the
// row loops and the cache test are scalar.
typedef float k2f2 __attribute__((ext_vector_type(2)));
template <bool FP16>
FFCV_DEV void k2_area_walk(const Epilogue &ep, const ResizePlan &P, const AreaTaps *atab, const uint8_t *rgb,
                           int pitch3, int xoff3, int r0, int oy0, int oy1, int sub, int dx0, uint32_t lutb,
                           char *ob) {
  const int half = (BAND + K2T / K2_COLS - 1) / (K2T / K2_COLS);  // rows per row group
  const int ya = __builtin_amdgcn_readfirstlane(oy0 + sub * half);
  const int yb = __builtin_amdgcn_readfirstlane(min(oy1, ya + half));
  const int out_w = ep.out_w;
  uint32_t xa[2], sh[2];  // a column's first tap: aligned byte offset in the row, byte shift
  k2f2 wk[3];             // tap k's weight for (dx0, dx0 + 1)
  {
    const AreaTaps t0 = area_taps(P.sw, P.scale_x, ep.src_x(dx0)), t1 = area_taps(P.sw, P.scale_x, ep.src_x(dx0 + 1));
    const uint32_t o0 = (uint32_t)(xoff3 + 3 * t0.lo), o1 = (uint32_t)(xoff3 + 3 * t1.lo);
    xa[0] = o0 & ~3u;
    sh[0] = o0 & 3u;
    xa[1] = o1 & ~3u;
    sh[1] = o1 & 3u;
#pragma unroll
    for (int k = 0; k < 3; k++)
      wk[k] = (k2f2){t0.lo + k <= t0.hi ? t0.w(t0.lo + k) : 0.f, t1.lo + k <= t1.hi ? t1.w(t1.lo + k) : 0.f};
  }
  // a column's three tap pixels are 9 consecutive bytes: three aligned dword
  // reads and v_alignbyte (misaligned LDS reads are several times slower)
  auto hsum = [&](int r, k2f2 B[3]) {
    const uint8_t *row = rgb + __mul24(r - r0, pitch3);
    uint32_t e[2][3];
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const uint32_t *qa = (const uint32_t *)(row + xa[j]);
      const uint32_t d0 = qa[0], d1 = qa[1], d2 = qa[2];
      e[j][0] = __builtin_amdgcn_alignbyte(d1, d0, sh[j]);
      e[j][1] = __builtin_amdgcn_alignbyte(d2, d1, sh[j]);
      e[j][2] = d2 >> (8 * sh[j]);
    }
    auto bx = [&](int i) {
      return (k2f2){(float)((e[0][i >> 2] >> (8 * (i & 3))) & 0xffu), (float)((e[1][i >> 2] >> (8 * (i & 3))) & 0xffu)};
    };
#pragma unroll
    for (int c = 0; c < 3; c++) {
      k2f2 b = bx(c) * wk[0];  // (0 + x == x for x >= 0: the reference's zeroed buf)
      b = b + bx(3 + c) * wk[1];
      b = b + bx(6 + c) * wk[2];
      B[c] = b;
    }
  };
  const bool cut0 = ep.in_cut(ep.cut_y, dx0), cut1 = ep.in_cut(ep.cut_y, dx0 + 1);
  int cr = -1;
  k2f2 Hc[3];
#pragma unroll
  for (int c = 0; c < 3; c++) Hc[c] = (k2f2){0.f, 0.f};
  for (int dy = ya; dy < yb; dy++) {
    const AreaTaps ty = atab[dy - oy0];
    k2f2 S[3];
    for (int r = ty.lo; r <= ty.hi; r++) {
      k2f2 H[3];
      if (r == cr) {
#pragma unroll
        for (int c = 0; c < 3; c++) H[c] = Hc[c];
      } else {
        hsum(r, H);
      }
      const k2f2 w = (k2f2){ty.w(r), ty.w(r)};
      if (r == ty.lo) {
#pragma unroll
        for (int c = 0; c < 3; c++) S[c] = w * H[c];
      } else {
#pragma unroll
        for (int c = 0; c < 3; c++) S[c] = S[c] + w * H[c];
      }
      if (r == ty.hi) {
#pragma unroll
        for (int c = 0; c < 3; c++) Hc[c] = H[c];
        cr = r;
      }
    }
    // cvRound + saturate_cast<uchar> of sums in [0, 255.5) (bytes times
    // weights summing to 1 up to a few float roundings): S + 1.5 * 2^23
    // rounds half-to-even into the float's low byte, one packed add per
    // column pair (the saturation never acts); only that byte is used
    uint32_t o[6];
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const k2f2 m = S[c] + (k2f2){12582912.0f, 12582912.0f};
      o[c] = ffcv_f2u_bits(m.x);
      o[3 + c] = ffcv_f2u_bits(m.y);
    }
    if ((cut0 || cut1) && dy >= ep.cut_y && dy < ep.cut_y + ep.cut_size) {
      if (cut0) {
        o[0] = ep.fill[0];
        o[1] = ep.fill[1];
        o[2] = ep.fill[2];
      }
      if (cut1) {
        o[3] = ep.fill[0];
        o[4] = ep.fill[1];
        o[5] = ep.fill[2];
      }
    }
    // the row's address is wave-uniform: scalar base + this thread's offset
    typedef __attribute__((address_space(1))) uint8_t gbyte_t;
    const uint64_t rb64 = (uint64_t)(uintptr_t)ob + (uint64_t)(uint32_t)dy * (uint32_t)((FP16 ? 6 : 3) * out_w);
    gbyte_t *orow = (gbyte_t *)(uintptr_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(rb64 >> 32)) << 32) |
                                           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)rb64));
    const uint32_t xoff = (uint32_t)((FP16 ? 6 : 3) * dx0);
    if (FP16) {  // LUT entry (v, c) at lutb + 2 v + 512 c (lut_ld)
      auto la = [&](uint32_t b) { return lutb + 2u * (b & 0xffu); };
      const uint32_t h0 = lut_ld(la(o[0]), 0), h1 = lut_ld(la(o[1]), 1), h2 = lut_ld(la(o[2]), 2);
      const uint32_t h3 = lut_ld(la(o[3]), 0), h4 = lut_ld(la(o[4]), 1), h5 = lut_ld(la(o[5]), 2);
      typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
      u32x3 w;
      w.x = h0 | (h1 << 16);
      w.y = h2 | (h3 << 16);
      w.z = h4 | (h5 << 16);
      __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x3 *)(orow + xoff));
    } else {
      __attribute__((address_space(1))) uint16_t *o16 =
          (__attribute__((address_space(1))) uint16_t *)(orow + xoff);  // low bytes of two values: v_perm
      o16[0] = (uint16_t)__builtin_amdgcn_perm(o[1], o[0], 0x0c0c0400u);
      o16[1] = (uint16_t)__builtin_amdgcn_perm(o[3], o[2], 0x0c0c0400u);
      o16[2] = (uint16_t)__builtin_amdgcn_perm(o[5], o[4], 0x0c0c0400u);
    }
  }
}
// One band of BAND output rows of image k (one per K2 workgroup; the
// band-loop form of round 4 was deleted in round 6: slower at the driver's
// launch sizes, equal at 400 steps).  Every barrier inside is reached by all threads;
// the only thread-level return follows the last one.
template <int MODE, bool FP16>
FFCV_DEV void k2_band(const JpegArgs &a, const int k, const int band, uint8_t *lds) {
  lds_u16_t *s_lut = (lds_u16_t *)lds;  // 768 entries (FP16), channel-major
  const int t = threadIdx.x;
  // ---- one round trip for everything that depends only on (k, band, t):
  // the record head, the LUT, this band's row taps, this thread's column
  // taps and the epilogue draws (see K2Rec)
  K2Rec R;
  R.load(a.info + k, t);
  constexpr int LU = (768 + K2T - 1) / K2T;
  uint16_t lv[LU];
  if (FP16) {
#pragma unroll
    for (int u = 0; u < LU; u++) lv[u] = u * K2T + t < 768 ? lut_src(a.p.lut, u * K2T + t) : (uint16_t)0;
  }
  const int band_rows_n = MODE == JM_RRC ? min(a.p.out_h - band * BAND, BAND) : 0;
  // K1 writes an image's tap table only when out_w + out_h fits K2_TAPS: a
  // larger output never reads it (and past the last image the index would
  // leave the allocation)
  const uint2 *ktaps = MODE == JM_RRC && a.taps && a.p.out_w + a.p.out_h <= K2_TAPS
                           ? a.taps + (uint64_t)k * K2_TAPS
                           : nullptr;
  uint2 rt_pre = make_uint2(0, 0);
  uint4 ct_pre = make_uint4(0, 0, 0, 0);
  if (ktaps) {
    if (t < band_rows_n) rt_pre = ktaps[a.p.out_w + band * BAND + t];
    if (2 * (t % K2_COLS) + 1 < a.p.out_w) ct_pre = *(const uint4 *)(ktaps + 2 * (t % K2_COLS));
  }
  const int cut_y0 = a.cut ? a.cut[2 * k] : 0, cut_x0 = a.cut ? a.cut[2 * k + 1] : 0;
  const int flip0 = a.flips ? a.flips[k] : 0;
  if (k == 0 && band == 0 && t == 0) {  // K1 is done: close its arena (see arena_before_k1)
    const unsigned long long top = a.arena_top[0];
    if (top) {
      a.arena_top[1] = top;
      a.arena_top[0] = 0;
    }
  }
  const ImgInfo I = k2_head(R);
  const int status = I.status;
  if (status == -1) return;  // raw sample (handled by the raw kernel)
  const int out_h = MODE == JM_FULL ? (int)a.samples[k].height : a.p.out_h;
  const int out_w = MODE == JM_FULL ? (int)a.samples[k].width : a.p.out_w;
  const int oy0 = band * BAND, oy1 = min(out_h, oy0 + BAND);
  if (oy0 >= out_h) return;
  char *ob = (char *)a.out + a.out_stride * k;
  const int esz = FP16 ? 2 : 1;
  if (status != FFCV_SAMPLE_OK) {  // zero-fill this band
    if (MODE == JM_RRC) {
      uint64_t row = (uint64_t)out_w * 3 * esz;
      for (uint64_t i = t; i < row * (oy1 - oy0); i += K2T) ob[row * oy0 + i] = 0;
    }
    return;
  }
  const uint8_t *planes = a.arena;
  const ColorGeom G = color_geom(I);
  const int ncomp = G.ncomp;
  GPlane gp[3];
#pragma unroll
  for (int c = 0; c < 3; c++) gp[c] = GPlane{planes + I.poff[c], I.stride[c]};
  if (MODE == JM_FULL) {
    uint8_t *o = (uint8_t *)ob;
    for (int i = t; i < (oy1 - oy0) * out_w; i += K2T) {
      int y = oy0 + i / out_w, x = i % out_w;
      int v[3];
      pixel_rgb(G, gp, y, x, v);
      uint8_t *d = o + ((uint64_t)y * out_w + x) * 3;
      d[0] = (uint8_t)v[0];
      d[1] = (uint8_t)v[1];
      d[2] = (uint8_t)v[2];
    }
    return;
  }
  if (FP16) {  // (loaded at the top)
#pragma unroll
    for (int u = 0; u < LU; u++)
      if (u * K2T + t < 768) s_lut[u * K2T + t] = lv[u];
  }
  const int ri = I.ri, rj = I.rj, rh = I.rh, rw = I.rw;
  const ResizePlan P = MODE == JM_RRC ? I.plan : make_plan(rw, rh, out_w, out_h);  // RRC: K1's plan
  const uint2 *taps = I.taps ? ktaps : nullptr;
  int r0, r1;
  band_rows(P, oy0, oy1, &r0, &r1);
  const int nrows = r1 - r0 + 1;
  const int step = rw * 3;
  // Epilogue parameters (flip, cutout) of this image
  Epilogue ep;
  ep.out_h = out_h;
  ep.out_w = out_w;
  ep.cut_size = a.cut ? a.p.cutout_size : 0;
  ep.cut_y = cut_y0;
  ep.cut_x = cut_x0;
  ep.flip = flip0;
  ep.cut_before_flip = a.p.cutout_fill[3];
  ep.fill[0] = a.p.cutout_fill[0];
  ep.fill[1] = a.p.cutout_fill[1];
  ep.fill[2] = a.p.cutout_fill[2];

  // ---- linear fast path (kind 3 with the SSE2 vertical body on every
  // element: every RRC crop that is upscaled along some axis at out_w 224).
  // LDS: [LUT][row taps][component tiles, dword rows][crop rows as RGBx
  // words].  Each thread owns one output column pair and walks its half of
  // the band's rows, keeping the two source rows' horizontal sums in
  // registers (resize.cpp HResizeLinear -> VResizeLinearVec_32s8u).
  // expansion factors 1 / 2 / 4 (every common subsampling): the tile bounds
  // below divide by shifts (a runtime x / ve compiles to a ~25-instruction
  // VALU sequence, twelve per workgroup); 3 takes the general path
  auto p2 = [](int x) { return x == 1 || x == 2 || x == 4; };
  const bool pow2 = p2(G.he[0]) && p2(G.ve[0]) && p2(G.he[1]) && p2(G.ve[1]) && p2(G.he[2]) && p2(G.ve[2]);
  // area fast path (round 6): INTER_AREA crops with both scales in [1, 2)
  // (every RRC crop larger than the output on both axes, up to 2x) of 4:2:0
  // images: the same tiles and colour pass, the crop rows kept as packed RGB
  // (3 bytes per pixel: 4-byte words would not fit a band's ~20 rows of up to
  // 256 px), then a column-pair walk with one cached row of horizontal sums
  // (as rrc_raw_kernel's area walk).  These bands took the general per-pixel
  // path before, ~3x the time of a linear band (r5z2_c3_k2_by_crop_perband.log).
  // (scale_x = 1 / (dw / sw) < 2 exactly when sw < 2 dw: integer tests keep
  // the f64 scales out of this condition, which cost 11 VGPRs)
  const bool area_fast = K2_AREA_FAST && P.kind == 2 && P.sw < 2 * P.dw && P.sh < 2 * P.dh && ncomp == 3 &&
                         !G.color_rgb && G.he[0] == 1 && G.ve[0] == 1 && G.he[1] == 2 && G.ve[1] == 2 &&
                         G.he[2] == 2 && G.ve[2] == 2 && G.cw[1] > 2 && G.cw[2] > 2;
  if (((P.kind == 3 && P.vec_end == 3 * out_w) || area_fast) && (out_w & 1) == 0 && out_w <= 2 * K2_COLS && pow2) {
    const int lut_b = FP16 ? 1536 : 0;
    LinTap *rtab = (LinTap *)(lds + lut_b);
    AreaTaps *atab = (AreaTaps *)(lds + lut_b);
    int ty0[3], tx0[3], trows[3], tpitch[3], toff[3];
    int need = lut_b + (area_fast ? (int)sizeof(AreaTaps) : (int)sizeof(LinTap)) * BAND;
#pragma unroll
    for (int c = 0; c < 3; c++) {
      if (c >= ncomp) {
        ty0[c] = tx0[c] = trows[c] = tpitch[c] = toff[c] = 0;
        continue;
      }
      const int he = G.he[c], ve = G.ve[c], hsh = he >> 1, vsh = ve >> 1;  // 1 / 2 / 4 -> 0 / 1 / 2
      int y0 = ((ri + r0) >> vsh) - (ve == 2 ? 1 : 0), y1 = ((ri + r1) >> vsh) + (ve == 2 ? 1 : 0);
      int x0 = (rj >> hsh) - (he == 2 ? 1 : 0), x1 = ((rj + rw - 1) >> hsh) + (he == 2 ? 1 : 0);
      y0 = max(y0, 0);
      x0 = max(x0, 0);
      y1 = min(y1, G.ch[c] - 1);
      x1 = min(x1, G.cw[c] - 1);
      ty0[c] = y0;
      tx0[c] = x0 & ~3;  // whole dwords of the plane row (rows are 8-byte aligned)
      trows[c] = y1 - y0 + 1;
      tpitch[c] = ((x1 + 4) & ~3) - tx0[c];
      toff[c] = need;
      need += trows[c] * tpitch[c];
    }
    const int rgb_off = need;
    // area: RGB rows from luma column Xb = 2 * (rj >> 1) (the colour pass's
    // first quad column), 12 bytes per chroma column pair, 4-byte aligned;
    // + 16 bytes for the walk's aligned reads past the last row's end
    const int pitch3 = 12 * (((((rj + rw - 1) >> 1) - (rj >> 1)) + 2) >> 1);
    need += area_fast ? nrows * pitch3 + 16 : nrows * rw * 4 + 4;  // linear: + a dummy word for off-crop pixels
    if (need <= K2_LDS) {
      K2_STOP_AT(1, a.out_stride != 77);  // diagnostics: the band's set-up (record, LUT, taps, tile bounds)
      uint32_t *rgbx = (uint32_t *)(lds + rgb_off);
      if (!area_fast && t < oy1 - oy0) {  // weights stored as the walk's multiplier operands, c << 8 (see hrow)
        LinTap lt = taps ? tap_unpack(rt_pre) : lin_tap(P.scale_y, P.inv_y, P.sh, oy0 + t);
        lt.c0 = (lt.c0 & 0xfff) << 8;
        lt.c1 = (lt.c1 & 0xfff) << 8;
        rtab[t] = lt;
      }
      TPlane tp[3];
      // tile staging: the first SU dwords per thread of every component are
      // loaded before any LDS write (one memory round trip, not one per
      // dword); row = i / wpr by a float reciprocal: exact while the +0.5
      // margin, 0.5 / (i + 0.5) relative, exceeds v_rcp_f32's 1 ulp plus the
      // product's rounding (i < 2^20; tiles here hold < 2^13 dwords)
      // Round 6: (float)i + 0.5 as t's float plus a constant, and the dword's
      // address as a 32-bit offset (24-bit multiply-add: tile offsets stay
      // below 2^24) from the component's scalar base (the saddr form) instead
      // of 64-bit address arithmetic per dword
      constexpr int SU = 4;
      uint32_t sv[3][SU];
      const float ft = (float)t + 0.5f;
      typedef const __attribute__((address_space(1))) uint8_t gu8_t;
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const int wpr = max(tpitch[c] >> 2, 1), n = trows[c] * (tpitch[c] >> 2);
        const float rwp = __builtin_amdgcn_rcpf((float)wpr);  // (1 ulp: far inside the +0.5 margin)
        gu8_t *src = (gu8_t *)(uintptr_t)(gp[c].p + (uint64_t)ty0[c] * gp[c].stride + tx0[c]);
        const uint32_t st = (uint32_t)gp[c].stride;
#pragma unroll
        for (int u = 0; u < SU; u++) {
          const int i = u * K2T + t;
          const int rr = (int)((ft + (float)(u * K2T)) * rwp), q = i - __mul24(rr, wpr);
          sv[c][u] = i < n ? *(const __attribute__((address_space(1))) uint32_t *)(src + (__umul24((uint32_t)rr, st) + 4u * (uint32_t)q)) : 0u;
        }
      }
#pragma unroll
      for (int c = 0; c < 3; c++) {
        uint32_t *tl = (uint32_t *)(lds + toff[c]);
        const int wpr = max(tpitch[c] >> 2, 1), n = trows[c] * (tpitch[c] >> 2);
#pragma unroll
        for (int u = 0; u < SU; u++)
          if (u * K2T + t < n) tl[u * K2T + t] = sv[c][u];
        const uint8_t *src = gp[c].p + (uint64_t)ty0[c] * gp[c].stride + tx0[c];
        const float rwp = __builtin_amdgcn_rcpf((float)wpr);
        for (int i = SU * K2T + t; i < n; i += K2T) {  // big tiles
          const int rr = (int)(((float)i + 0.5f) * rwp), q = i - __mul24(rr, wpr);
          tl[i] = *(const uint32_t *)(src + (uint64_t)rr * gp[c].stride + 4 * q);
        }
        tp[c] = TPlane{(const uint8_t *)tl, ty0[c], tx0[c], tpitch[c]};
      }
      // (after the tiles: its f64 arithmetic would raise the register peak
      // while the tile loads are in flight)
      if (area_fast && t < oy1 - oy0) atab[t] = area_taps(P.sh, P.scale_y, oy0 + t);
      __syncthreads();
      K2_STOP_AT(2, a.out_stride != 77);  // diagnostics: + the plane tiles
      const int Y0 = ri + r0, Y1 = ri + r1, X0 = rj, X1 = rj + rw - 1;
      if (ncomp == 3 && !G.color_rgb && G.he[0] == 1 && G.ve[0] == 1 && G.he[1] == 2 && G.ve[1] == 2 &&
          G.he[2] == 2 && G.ve[2] == 2 && G.cw[1] > 2 && G.cw[2] > 2) {  // (every area_fast band)
        // 4:2:0 (jdsample.c h2v2_fancy_upsample, as upsample_quad_h2v2): each
        // thread owns a pair of adjacent chroma columns (C, C + 1) and walks
        // every ng-th chroma row of the band.  Column clamps, edge terms and
        // offsets are computed once per thread; per row the 3 x 4 chroma
        // neighbourhood of the two quads is read once per plane and its
        // vertical sums (3 * centre + above / below) are shared by both quads.
        // Pixels outside the crop go to a dummy LDS word (branch-free).
        const int R0 = Y0 >> 1, R1 = Y1 >> 1, C0 = X0 >> 1, C1 = X1 >> 1;
        const int npairs = (C1 - C0 + 2) >> 1;
        const int ps = min(npairs, K2T);  // pairs per sweep of the workgroup
        const float rp = __builtin_amdgcn_rcpf((float)ps);
        // ng row groups; t = g * ps + pair (quotients by a float reciprocal:
        // exact for these small operands, as in the tile staging)
        const int ng = (int)(((float)K2T + 0.5f) * rp);
        const int g = (int)(((float)t + 0.5f) * rp);
        if (g < ng)
        for (int pr = t - __mul24(g, ps); pr < npairs; pr += ps) {
          const int C = C0 + 2 * pr;
          // plane columns of the two quads' neighbourhoods (clamped like
          // upsample_quad_h2v2; the fourth is unused without a second quad)
          const int cw = G.cw[1], ch = G.ch[1];
          const int xm = max(C - 1, 0) - tp[1].c0, x0 = C - tp[1].c0;
          const int x1 = min(C + 1, cw - 1) - tp[1].c0, x2 = min(C + 2, min(C1 + 1, cw - 1)) - tp[1].c0;
          // luma columns 2C .. 2C + 3: inside the crop?  (reads clamped into it)
          const int X = 2 * C;
          bool vx[4];
          int lx[4];
#pragma unroll
          for (int j = 0; j < 4; j++) {
            vx[j] = X + j >= X0 && X + j <= X1;
            lx[j] = min(max(X + j, X0), X1) - tp[0].c0;
          }
          uint32_t *dummy = rgbx + nrows * rw;
          for (int R = R0 + g; R <= R1; R += ng) {
            const int ru = max(R - 1, 0), rd = min(R + 1, ch - 1);
            int qb[2][8];  // [plane][quad u: C's q0..q3, then C + 1's]
#pragma unroll
            for (int pl = 0; pl < 2; pl++) {
              const uint8_t *b = tp[1 + pl].p;
              const int pitch = tp[1 + pl].pitch, ty = tp[1 + pl].r0;
              const uint8_t *rm = b + __mul24(R - ty, pitch), *ra = b + __mul24(ru - ty, pitch),
                            *rb = b + __mul24(rd - ty, pitch);
              const int mm = rm[xm], m0 = rm[x0], m1 = rm[x1], m2 = rm[x2];
              // vertical sums above (T) and below (B) for columns xm, x0, x1, x2
              const int Tm = 3 * mm + ra[xm], T0 = 3 * m0 + ra[x0], T1 = 3 * m1 + ra[x1], T2 = 3 * m2 + ra[x2];
              const int Bm = 3 * mm + rb[xm], B0 = 3 * m0 + rb[x0], B1 = 3 * m1 + rb[x1], B2 = 3 * m2 + rb[x2];
              qb[pl][0] = (3 * T0 + Tm + 8) >> 4;
              qb[pl][1] = (3 * T0 + T1 + 7) >> 4;
              qb[pl][2] = (3 * B0 + Bm + 8) >> 4;
              qb[pl][3] = (3 * B0 + B1 + 7) >> 4;
              qb[pl][4] = (3 * T1 + T0 + 8) >> 4;
              qb[pl][5] = (3 * T1 + T2 + 7) >> 4;
              qb[pl][6] = (3 * B1 + B0 + 8) >> 4;
              qb[pl][7] = (3 * B1 + B2 + 7) >> 4;
            }
            if (area_fast) {  // four packed RGB pixels per row: 3 words at byte 12 * pr of the row
#pragma unroll
              for (int dy = 0; dy < 2; dy++) {
                const int Y = 2 * R + dy;
                const uint8_t *ly = tp[0].p + __mul24(min(max(Y, Y0), Y1) - tp[0].r0, tp[0].pitch);
                uint32_t px[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                  const int u = (j >> 1) * 4 + dy * 2 + (j & 1);
                  int v[3];
                  ycc_rgb(ly[lx[j]], qb[0][u], qb[1][u], v);
                  px[j] = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16);
                }
                if (Y >= Y0 && Y <= Y1) {
                  uint32_t *d = rgbx + __mul24(Y - Y0, pitch3 >> 2) + 3 * pr;
                  d[0] = px[0] | (px[1] << 24);
                  d[1] = (px[1] >> 8) | (px[2] << 16);
                  d[2] = (px[2] >> 16) | (px[3] << 8);
                }
              }
              continue;
            }
#pragma unroll
            for (int dy = 0; dy < 2; dy++) {
              const int Y = 2 * R + dy;
              const bool vy = Y >= Y0 && Y <= Y1;
              const uint8_t *ly = tp[0].p + __mul24(min(max(Y, Y0), Y1) - tp[0].r0, tp[0].pitch);
              uint32_t *orow = rgbx + __mul24(Y - Y0, rw) - X0;
#pragma unroll
              for (int j = 0; j < 4; j++) {
                const int u = (j >> 1) * 4 + dy * 2 + (j & 1);  // quad, then its q index
                int v[3];
                ycc_rgb(ly[lx[j]], qb[0][u], qb[1][u], v);
                uint32_t *d = vy && vx[j] ? orow + X + j : dummy;
                *d = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16);
              }
            }
          }
        }
      } else {
        for (int i = t; i < nrows * rw; i += K2T) {
          const int yy = i / rw, x = i - yy * rw;
          int v[3];
          pixel_rgb(G, tp, Y0 + yy, X0 + x, v);
          rgbx[i] = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16);
        }
      }
      __syncthreads();
      K2_STOP_AT(3, a.out_stride != 77);  // diagnostics: + the colour pass
      const int tx = t % K2_COLS, sub = t / K2_COLS;
      if (tx >= out_w / 2) return;
      const int dx0 = 2 * tx;
      if (area_fast) {
        k2_area_walk<FP16>(ep, P, atab, (const uint8_t *)rgbx, pitch3, 3 * (rj - 2 * (rj >> 1)), r0, oy0, oy1, sub,
                           dx0, lut_base(s_lut), ob);
        return;
      }
      LinTap l0, l1;
      if (taps) {  // K1's table (flip applied): both columns in one 16-byte load (at the top)
        const uint4 q = ct_pre;
        l0 = tap_unpack(make_uint2(q.x, q.y));
        l1 = tap_unpack(make_uint2(q.z, q.w));
      } else {
        l0 = lin_tap(P.scale_x, P.inv_x, P.sw, ep.src_x(dx0));
        l1 = lin_tap(P.scale_x, P.inv_x, P.sw, ep.src_x(dx0 + 1));
      }
      // a border tap (src[s] * 2048) as the same two-tap form with weights
      // (2048, 0) on (s, s + 1): branch-free, identical sums
      const int a0w = l0.border ? 2048 : l0.c0, b0w = l0.border ? 0 : l0.c1;
      const int a1w = l1.border ? 2048 : l1.c0, b1w = l1.border ? 0 : l1.c1;
      // horizontal pass of crop row r for both columns: sat_s16(h >> 4) per
      // channel.  The saturations of this walk never act (so they are not
      // computed): weights are in [0, 2048] with c0 + c1 <= 2049 (linear_coef
      // rounds each), so 0 <= h >> 4 <= 255 * 2049 >> 4 = 32655 and the
      // vertical sum m0 + m1 <= 32655 * 2049 >> 16 = 1020, (1020 + 2) >> 2 = 255.
      // The rows keep (h >> 4) << 8 (< 2^23), so VResizeLinearVec's
      // (h * c) >> 16 is one 24-bit high multiply by c << 8 (< 2^20):
      // mulhi_u24(h << 8, c << 8) = (h * c * 2^16) >> 32.
      // On gfx950 every multiply, bit-field extract and 3-operand integer
      // form issues in 4 cycles per wave against 2 for add / shift / and
      // (tools/op_rate), so the pair of a channel's two source samples is
      // gathered by one v_perm_b32 as u16 halves and weighted by one
      // v_dot2_u32_u16 with the weights pre-scaled by 16: dot = 16 h, and
      // (h >> 4) << 8 = dot & 0x7fff00 (10 cycles per value instead of 22).
      const uint32_t w0 = ((uint32_t)a0w << 4) | ((uint32_t)b0w << 20), w1 = ((uint32_t)a1w << 4) | ((uint32_t)b1w << 20);
      const uint32_t so0 = 4u * (uint32_t)l0.s, so1 = 4u * (uint32_t)l1.s;  // byte offsets in a row
      auto hrow = [&](int r, uint32_t H[6]) {
        const uint32_t *row = rgbx + __mul24(r - r0, rw);
        // words s and s + 1 as one ds_read2 per column (a border tap's second
        // word has weight 0: at the crop's right edge it is the next row's
        // first word or, in the last row, the dummy word)
        const uint32_t *e0 = (const uint32_t *)((const uint8_t *)row + so0), *e1 = (const uint32_t *)((const uint8_t *)row + so1);
        const uint32_t p0 = e0[0], q0 = e0[1];
        const uint32_t p1 = e1[0], q1 = e1[1];
#pragma unroll
        for (int c = 0; c < 3; c++) {
          // bytes [p.c, 0, q.c, 0]: v_perm_b32 selector c | 0x0c << 8 | (4 + c) << 16 | 0x0c << 24
          const uint32_t sel = (uint32_t)c | 0x0c00u | ((uint32_t)(4 + c) << 16) | 0x0c000000u;
          H[c] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, __builtin_amdgcn_perm(q0, p0, sel)),
                                        __builtin_bit_cast(u16x2_t, w0), 0u, false) & 0x7fff00u;
          H[3 + c] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2_t, __builtin_amdgcn_perm(q1, p1, sel)),
                                            __builtin_bit_cast(u16x2_t, w1), 0u, false) & 0x7fff00u;
        }
      };
      auto mulhi24 = [](uint32_t x, uint32_t y) -> uint32_t {  // x, y < 2^24: v_mul_hi_u32_u24
        return (uint32_t)(((uint64_t)(x & 0xffffffu) * (y & 0xffffffu)) >> 32);
      };
      // cutout: which of this thread's two columns lie in the square (tested
      // once; a row tests its own range)
      const bool cut0 = ep.in_cut(ep.cut_y, dx0), cut1 = ep.in_cut(ep.cut_y, dx0 + 1);
      const uint32_t lq = FP16 ? 2u + 2u * lut_base(s_lut) : 2u;  // (lut_q)
      uint32_t qfill[3];  // the cutout fill as lut_q's result
      for (int c = 0; c < 3; c++) qfill[c] = FP16 ? lut_base(s_lut) + 2u * ep.fill[c] : ep.fill[c];
      const int half = (BAND + K2T / K2_COLS - 1) / (K2T / K2_COLS);  // rows per row group
      // (a row group is two whole waves: its rows are wave-uniform, so the
      // per-row tap read, cutout test and row changes are scalar)
      const int ya = __builtin_amdgcn_readfirstlane(oy0 + sub * half);
      const int yb = __builtin_amdgcn_readfirstlane(min(oy1, ya + half));
      int ca = -1, cb = -1;
      uint32_t HA[6], HB[6];
      for (int dy = ya; dy < yb; dy++) {
        const LinTap ly = rtab[dy - oy0];
        const int ra = min(max(ly.s, 0), P.sh - 1), rb = min(max(ly.s + 1, 0), P.sh - 1);
        if (ra != ca) {
          if (ra == cb) {
#pragma unroll
            for (int i = 0; i < 6; i++) HA[i] = HB[i];
          } else {
            hrow(ra, HA);
          }
          ca = ra;
        }
        if (rb != cb) {
          hrow(rb, HB);
          cb = rb;
        }
        uint32_t o[6];
        const uint32_t c0 = ly.c0, c1 = ly.c1;  // (pre-scaled in rtab)
#pragma unroll
        for (int i = 0; i < 6; i++)  // (sat_s16(m0 + m1) + 2) >> 2, no saturation (see hrow); FP16: its LUT address
          o[i] = lut_q<FP16>(mulhi24(HA[i], c0) + mulhi24(HB[i], c1), lq);
        if ((cut0 || cut1) && dy >= ep.cut_y && dy < ep.cut_y + ep.cut_size) {
          if (cut0) {
            o[0] = qfill[0];
            o[1] = qfill[1];
            o[2] = qfill[2];
          }
          if (cut1) {
            o[3] = qfill[0];
            o[4] = qfill[1];
            o[5] = qfill[2];
          }
        }
#if K2_SADDR_STORE
        // (round 6) the row's address is wave-uniform (dy is): scalar base +
        // this thread's fixed 32-bit offset (the store's saddr form), no
        // 64-bit address arithmetic per row
        typedef __attribute__((address_space(1))) uint8_t gbyte_t;
        const uint64_t rb64 = (uint64_t)(uintptr_t)ob + (uint64_t)(uint32_t)dy * (uint32_t)(3 * esz * out_w);
        gbyte_t *orow = (gbyte_t *)(uintptr_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(rb64 >> 32)) << 32) |
                                               (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)rb64));
        const uint32_t xoff = (uint32_t)(3 * esz * dx0);
#else
        const uint64_t p0 = (uint64_t)dy * out_w + dx0;
#endif
        if (FP16) {
          const uint32_t h0 = lut_ld(o[0], 0), h1 = lut_ld(o[1], 1), h2 = lut_ld(o[2], 2);
          const uint32_t h3 = lut_ld(o[3], 0), h4 = lut_ld(o[4], 1), h5 = lut_ld(o[5], 2);
          typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));  // 12-byte group, 4-byte aligned
          u32x3 w;
          w.x = h0 | (h1 << 16);
          w.y = h2 | (h3 << 16);
          w.z = h4 | (h5 << 16);
          // streaming output: non-temporal (measured +2.7% C3 over plain stores)
#if K2_SADDR_STORE
          __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x3 *)(orow + xoff));
#else
          __builtin_nontemporal_store(w, (u32x3 *)((uint16_t *)ob + p0 * 3));
#endif
        } else {
#if K2_SADDR_STORE
          __attribute__((address_space(1))) uint16_t *o16 = (__attribute__((address_space(1))) uint16_t *)(orow + xoff);
#else
          uint16_t *o16 = (uint16_t *)((uint8_t *)ob + p0 * 3);
#endif
          o16[0] = (uint16_t)(o[0] | (o[1] << 8));
          o16[1] = (uint16_t)(o[2] | (o[3] << 8));
          o16[2] = (uint16_t)(o[4] | (o[5] << 8));
        }
      }
      return;
    }
  }
  // diagnostics (K1's stamp buffer, slot 11): bands of this image that take
  // the general path below
  if (a.dbg && t == 0) atomicAdd((unsigned long long *)(a.dbg + (uint64_t)k * 16 + 11), 1ull);
  // LDS: [LUT][column + row taps][component tiles][RGB rows].  The taps of
  // the band's rows and of every output column are computed once per
  // workgroup; the tiles cover every plane sample the band's upsampling
  // reads, so the colour pass runs from LDS.
  const int tap_b = (P.kind == 2 ? (int)sizeof(AreaTaps) : (P.kind == 3 ? (int)sizeof(LinTap) : 0)) * (out_w + BAND);
  const int lut_b = (FP16 ? 1536 : 0) + ((tap_b + 15) & ~15);
  AreaTaps *atab = (AreaTaps *)(lds + (FP16 ? 1536 : 0));
  LinTap *ltab = (LinTap *)atab;
  int ty0[3], tx0[3], trows[3], tcols[3], toff[3];
  int need = lut_b;
#pragma unroll
  for (int c = 0; c < 3; c++) {  // (unrolled: no dynamically indexed arrays)
    if (c >= ncomp) {
      ty0[c] = tx0[c] = trows[c] = tcols[c] = toff[c] = 0;
      continue;
    }
    const int he = G.he[c], ve = G.ve[c];
    int y0 = (ri + r0) / ve - (ve == 2 ? 1 : 0), y1 = (ri + r1) / ve + (ve == 2 ? 1 : 0);
    int x0 = rj / he - (he == 2 ? 1 : 0), x1 = (rj + rw - 1) / he + (he == 2 ? 1 : 0);
    y0 = max(y0, 0);
    x0 = max(x0, 0);
    y1 = min(y1, G.ch[c] - 1);
    x1 = min(x1, G.cw[c] - 1);
    ty0[c] = y0;
    tx0[c] = x0;
    trows[c] = y1 - y0 + 1;
    tcols[c] = x1 - x0 + 1;
    toff[c] = need;
    need += (trows[c] * tcols[c] + 15) & ~15;
  }
  const int roi_off = need;
  need += nrows * step;
  const bool tiled = need <= K2_LDS;
  const bool staged = tiled || lut_b + nrows * step <= K2_LDS;  // (tap tables fit: see tabs)
  uint8_t *roi = lds + (tiled ? roi_off : lut_b);
  // Bands too wide for LDS stage their rows in the image's rgb slot at their
  // absolute crop-row position; rows shared with a neighbouring band are
  // written with identical bytes by both.
  uint8_t *groi = a.arena + I.rgb_off;
  uint8_t *dst = staged ? roi : groi + (uint64_t)r0 * step;
  const bool tabs = tap_b > 0 && lut_b <= K2_LDS / 2;
  if (tabs) {  // [0, out_w): columns, [out_w, out_w + rows): the band's rows
    for (int i = t; i < out_w + (oy1 - oy0); i += K2T) {
      if (P.kind == 2)
        atab[i] = i < out_w ? area_taps(P.sw, P.scale_x, i) : area_taps(P.sh, P.scale_y, oy0 + i - out_w);
      else
        ltab[i] = i < out_w ? lin_tap(P.scale_x, P.inv_x, P.sw, i) : lin_tap(P.scale_y, P.inv_y, P.sh, oy0 + i - out_w);
    }
  }
  if (tiled) {
    TPlane tp[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
      uint8_t *tl = lds + toff[c];
      const int cols = tcols[c], n = trows[c] * cols;
      const uint8_t *src = gp[c].p + (uint64_t)ty0[c] * gp[c].stride + tx0[c];
      for (int i = t; i < n; i += K2T) {
        const int rr = i / cols, cc = i - rr * cols;
        tl[rr * cols + cc] = src[(uint64_t)rr * gp[c].stride + cc];
      }
      tp[c] = TPlane{tl, ty0[c], tx0[c], cols};
    }
    __syncthreads();
    const bool q420 = ncomp == 3 && !G.color_rgb && G.he[0] == 1 && G.ve[0] == 1 && G.he[1] == 2 &&
                      G.ve[1] == 2 && G.he[2] == 2 && G.ve[2] == 2 && G.cw[1] > 2 && G.cw[2] > 2;
    if (q420) {  // one thread per chroma sample: a 2x2 quad of pixels
      const int Y0 = ri + r0, Y1 = ri + r1, X0 = rj, X1 = rj + rw - 1;
      const int R0 = Y0 >> 1, C0 = X0 >> 1, qcols = (X1 >> 1) - C0 + 1;
      const int nq = ((Y1 >> 1) - R0 + 1) * qcols;
      for (int i = t; i < nq; i += K2T) {
        const int qr = i / qcols, R = R0 + qr, C = C0 + (i - qr * qcols);
        int cb[4], cr[4];
        upsample_quad_h2v2(tp[1], G.cw[1], G.ch[1], R, C, cb);
        upsample_quad_h2v2(tp[2], G.cw[2], G.ch[2], R, C, cr);
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int Y = 2 * R + (u >> 1), X = 2 * C + (u & 1);
          if (Y < Y0 || Y > Y1 || X < X0 || X > X1) continue;
          int v[3];
          ycc_rgb(tp[0].at(Y, X), cb[u], cr[u], v);
          uint8_t *d = dst + (Y - Y0) * step + (X - X0) * 3;
          d[0] = (uint8_t)v[0];
          d[1] = (uint8_t)v[1];
          d[2] = (uint8_t)v[2];
        }
      }
    } else {
      for (int i = t; i < nrows * rw; i += K2T) {
        int yy = i / rw, x = i - yy * rw;
        int v[3];
        pixel_rgb(G, tp, ri + r0 + yy, rj + x, v);
        uint8_t *d = dst + yy * step + x * 3;
        d[0] = (uint8_t)v[0];
        d[1] = (uint8_t)v[1];
        d[2] = (uint8_t)v[2];
      }
    }
  } else {
    for (int i = t; i < nrows * rw; i += K2T) {
      int yy = i / rw, x = i - yy * rw;
      int v[3];
      pixel_rgb(G, gp, ri + r0 + yy, rj + x, v);
      uint8_t *d = dst + (uint64_t)yy * step + x * 3;
      d[0] = (uint8_t)v[0];
      d[1] = (uint8_t)v[1];
      d[2] = (uint8_t)v[2];
    }
  }
  // Separable linear (kind 3): OpenCV's horizontal pass depends only on the
  // source row, so each (row, column) tap pair is computed once per band and
  // kept as the saturated int16 (h >> 4) the vertical SIMD body consumes
  // (resize.cpp VResizeLinearVec_32s8u).  Columns in the scalar tail
  // (>= vec_end) keep the per-pixel path.
  const int hoff = (((tiled ? roi_off : lut_b) + nrows * step) + 15) & ~15;
  const bool sep = P.kind == 3 && staged && tabs && hoff + nrows * out_w * 8 <= K2_LDS;
  uint2 *H = (uint2 *)(lds + hoff);
  __syncthreads();
  if (sep) {
    for (int i = t; i < nrows * out_w; i += K2T) {
      const int rr = i / out_w, cx = i - rr * out_w;
      const LinTap lx = ltab[cx];
      const uint8_t *q = roi + rr * step + lx.s * 3;
      int hv[3];
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const int h = lx.border ? q[c] * 2048 : q[c] * lx.c0 + q[c + 3] * lx.c1;
        hv[c] = sat_s16i(h >> 4);
      }
      H[i] = make_uint2((uint32_t)(hv[0] & 0xffff) | ((uint32_t)hv[1] << 16), (uint32_t)(hv[2] & 0xffff));
    }
    __syncthreads();
  }
  LdsRoi lr{roi, r0, step};
  // resize_area_lds reads up to 5 bytes past the staged rows
  const bool pad8 = (int)(roi - lds) + nrows * step + 8 <= K2_LDS;
  RoiSrc gr{groi, (uint64_t)step};
  auto px = [&](int dy, int dx, int v[3]) {
    if (ep.in_cut(dy, dx)) {
      v[0] = ep.fill[0];
      v[1] = ep.fill[1];
      v[2] = ep.fill[2];
    } else if (sep && ep.src_x(dx) * 3 + 2 < P.vec_end) {
      const int cx = ep.src_x(dx);
      const LinTap ly = ltab[out_w + dy - oy0];
      const int ra = min(max(ly.s, 0), P.sh - 1) - r0, rb = min(max(ly.s + 1, 0), P.sh - 1) - r0;
      const uint2 A = H[ra * out_w + cx], Bv = H[rb * out_w + cx];
      const int a0[3] = {(int16_t)(A.x & 0xffff), (int16_t)(A.x >> 16), (int16_t)(A.y & 0xffff)};
      const int b0[3] = {(int16_t)(Bv.x & 0xffff), (int16_t)(Bv.x >> 16), (int16_t)(Bv.y & 0xffff)};
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const int m0 = __mul24(a0[c], ly.c0) >> 16, m1 = __mul24(b0[c], ly.c1) >> 16;
        v[c] = sat_u8i((sat_s16i(m0 + m1) + 2) >> 2);
      }
    } else if (staged && tabs) {
      const int cx = ep.src_x(dx);
      if (P.kind == 2 && pad8)  // (aligned reads: see resize_area_lds)
        resize_area_lds(lr, atab[cx], atab[out_w + dy - oy0], v);
      else if (P.kind == 2)
        resize_area(lr, atab[cx], atab[out_w + dy - oy0], v);
      else
        resize_linear(P, lr, cx, ltab[cx], ltab[out_w + dy - oy0], v);
    } else if (staged) {
      resize_pixel(P, lr, dy, ep.src_x(dx), v);
    } else {
      resize_pixel(P, gr, dy, ep.src_x(dx), v);
    }
  };
  // pixel pairs: 12 bytes (fp16) / 6 bytes (u8) per thread, 4-/2-byte
  // aligned when rows and samples start aligned; single pixels otherwise
  const bool pairs = (out_w & 1) == 0 && (a.out_stride & 3) == 0;
  const int per = pairs ? 2 : 1;
  const int hw = out_w / per;
  const int npx = (oy1 - oy0) * hw;
  for (int i = t; i < npx; i += K2T) {
    const int dy = oy0 + i / hw, dx = per * (i % hw);
    const bool two = pairs;
    int v[3], u[3];
    px(dy, dx, v);
    if (two) px(dy, dx + 1, u);
    const uint64_t p0 = (uint64_t)dy * out_w + dx;
    if (FP16) {
      uint16_t h0 = lut_at(s_lut, v[0], 0), h1 = lut_at(s_lut, v[1], 1), h2 = lut_at(s_lut, v[2], 2);
      uint16_t *o = (uint16_t *)ob + p0 * 3;
      if (two) {
        uint16_t h3 = lut_at(s_lut, u[0], 0), h4 = lut_at(s_lut, u[1], 1), h5 = lut_at(s_lut, u[2], 2);
        uint32_t *o32 = (uint32_t *)o;  // p0 even -> 12-byte aligned group
        o32[0] = h0 | ((uint32_t)h1 << 16);
        o32[1] = h2 | ((uint32_t)h3 << 16);
        o32[2] = h4 | ((uint32_t)h5 << 16);
      } else {
        o[0] = h0;
        o[1] = h1;
        o[2] = h2;
      }
    } else {
      uint8_t *o = (uint8_t *)ob + p0 * 3;
      if (two) {
        uint16_t *o16 = (uint16_t *)o;
        o16[0] = (uint16_t)(v[0] | (v[1] << 8));
        o16[1] = (uint16_t)(v[2] | (u[0] << 8));
        o16[2] = (uint16_t)(u[1] | (u[2] << 8));
      } else {
        o[0] = (uint8_t)v[0];
        o[1] = (uint8_t)v[1];
        o[2] = (uint8_t)v[2];
      }
    }
  }
}

template <int MODE, bool FP16>
__global__ void __launch_bounds__(K2T) __attribute__((amdgpu_waves_per_eu(K2_WPE))) jpeg_color_resize_kernel(JpegArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  k2_band<MODE, FP16>(a, (int)blockIdx.y, (int)blockIdx.x, lds);
}

// ---------------------------------------------------------------- ctx -----
struct ffcv_jpeg_ctx {
  uint64_t *dbg;
  int diag_only;    // diagnostics (ffcv_jpeg_set_diag): kernels a launch runs
  int max_batch;
  uint32_t max_h, max_w;
  uint64_t max_bytes;
  uint8_t *arena;  // per-launch scratch, bump-allocated per image by K1
  uint64_t arena_bytes;
  unsigned long long *arena_top;  // [0] bump counter, [1] high water of the last launch K2 closed
  bool arena_zero;  // [0] is 0 at the stream's tail: the last launch ran K2, which zeroes it
  ImgInfo *info;
  uint2 *taps;
  uint8_t *gtab;
  uint32_t *k1_order;  // max_batch slots (k1_order_kernel); used when k1_sorted
  bool k1_sorted;
  uint64_t gtab_slot;
  uint32_t *eidx;  // entropy index (caller-owned), or NULL
  uint64_t eidx_n;
  // per-kernel timing (ffcv_jpeg_set_timing): 4 events per launch recorded on
  // the launch's stream before K1, after K1, after K1b and after K2
  hipEvent_t *tev;
  int tev_cap, tev_n;
};

static uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

static void free_timing(ffcv_jpeg_ctx *c) {
  for (int i = 0; i < 4 * c->tev_cap; i++) (void)hipEventDestroy(c->tev[i]);
  delete[] c->tev;
  c->tev = nullptr;
  c->tev_cap = c->tev_n = 0;
}

static void free_ctx(ffcv_jpeg_ctx *c) {
  free_timing(c);
  (void)hipFree(c->arena);
  (void)hipFree(c->arena_top);
  (void)hipFree(c->info);
  (void)hipFree(c->taps);
  (void)hipFree(c->gtab);
  (void)hipFree(c->k1_order);
  delete c;
}

extern "C" {

uint64_t ffcv_jpeg_scratch_bound(uint32_t height, uint32_t width, uint64_t nbytes) {
  // every region alloc_scratch can take for an image of this size, whatever
  // its crop, sampling and MCU padding (hmax, vmax <= 4; <= 10 blocks per MCU)
  const uint64_t blocks = 3 * ((uint64_t)(width + 7) / 8 + 4) * ((uint64_t)(height + 7) / 8 + 4);
  return align_up(nbytes + 64, 256) + align_up(blocks * 128, 256) + align_up(blocks * 2, 256) +
         align_up(blocks * 64, 256) + align_up((uint64_t)height * width * 3, 256);
}

int ffcv_jpeg_create_arena(ffcv_jpeg_ctx **out, int max_batch, uint32_t max_height, uint32_t max_width,
                           uint64_t max_bytes, uint64_t arena_bytes) {
  if (!out || max_batch <= 0 || max_height == 0 || max_width == 0 || max_height > 65535 ||
      max_width > 65535 || max_bytes == 0) {
    ffcv::set_error("ffcv_jpeg_create: invalid arguments");
    return FFCV_EINVAL;
  }
  ffcv_jpeg_ctx *c = new ffcv_jpeg_ctx();
  c->max_batch = max_batch;
  c->diag_only = 7;
  {
    const char *o = getenv("FFCV_K1_ORDER");  // size-grouped K1 workgroups (A/B knob: 0 turns it off)
    c->k1_sorted = !o || atoi(o) != 0;
  }
  c->max_h = max_height;
  c->max_w = max_width;
  c->max_bytes = max_bytes;
  // default: room for max_batch images of the maximum size (never exhausted)
  c->arena_bytes = arena_bytes ? arena_bytes
                               : (uint64_t)max_batch * ffcv_jpeg_scratch_bound(max_height, max_width, max_bytes);
  c->gtab_slot = align_up(sizeof(JTables), 256);
  hipError_t e;
  if ((e = hipMalloc(&c->arena, c->arena_bytes)) != hipSuccess ||
      (e = hipMalloc(&c->arena_top, 2 * sizeof(unsigned long long))) != hipSuccess ||
      (e = hipMemset(c->arena_top, 0, 2 * sizeof(unsigned long long))) != hipSuccess ||
      (e = hipMalloc(&c->info, sizeof(ImgInfo) * max_batch)) != hipSuccess ||
      (e = hipMalloc(&c->taps, sizeof(uint2) * K2_TAPS * max_batch)) != hipSuccess ||
      (e = hipMalloc(&c->gtab, c->gtab_slot * max_batch)) != hipSuccess ||
      (e = hipMalloc(&c->k1_order, sizeof(uint32_t) * max_batch)) != hipSuccess ||
      // the memset above runs on the null stream, which the caller's
      // non-blocking streams do not wait for: finish it here (a first launch
      // on another stream read a stale counter left in reused memory and
      // failed every image TOO_LARGE)
      (e = hipStreamSynchronize(nullptr)) != hipSuccess) {
    int rc = ffcv::check_hip(e, "ffcv_jpeg_create: hipMalloc");
    free_ctx(c);
    return rc;
  }
  c->arena_zero = false;  // the first launch also zeroes the counter, on its own stream
  *out = c;
  return FFCV_OK;
}

int ffcv_jpeg_create(ffcv_jpeg_ctx **out, int max_batch, uint32_t max_height, uint32_t max_width,
                     uint64_t max_bytes) {
  return ffcv_jpeg_create_arena(out, max_batch, max_height, max_width, max_bytes, 0);
}

// Diagnostic hook (not in the public header): per-image phase stamps
// (wall_clock64, 100 MHz) into dbg[B][16]; NULL disables.
int ffcv_jpeg_set_debug(ffcv_jpeg_ctx *c, uint64_t *dbg) {
  if (!c) return FFCV_EINVAL;
  c->dbg = dbg;
  return FFCV_OK;
}

// Diagnostic hook (not in the public header): which kernels a decode launch
// runs (bit 0 = K1, bit 1 = the IDCT kernel, bit 2 = K2; timing of one kernel
// re-run on the previous launch's scratch) and K2 timing-only flags.  Set once per context, never
// read from the environment on the launch path.
int ffcv_jpeg_set_diag(ffcv_jpeg_ctx *c, int only, int k2flags) {
  // (k2flags: the K2 timing-only switches of rounds 1-4 are gone from the
  // product kernels; only 0 is accepted)
  if (!c || k2flags != 0) return FFCV_EINVAL;
  c->diag_only = only ? only : 7;
  return FFCV_OK;
}

int ffcv_jpeg_set_timing(ffcv_jpeg_ctx *c, int max_launches) {
  if (!c || max_launches < 0) {
    ffcv::set_error("ffcv_jpeg_set_timing: invalid arguments");
    return FFCV_EINVAL;
  }
  free_timing(c);
  if (!max_launches) return FFCV_OK;
  c->tev = new hipEvent_t[4 * (size_t)max_launches]();
  for (int i = 0; i < 4 * max_launches; i++) {
    hipError_t e = hipEventCreate(&c->tev[i]);
    if (e != hipSuccess) {
      c->tev_cap = i / 4;  // destroy what was made (whole sets, then the partial one)
      for (int j = 4 * c->tev_cap; j < i; j++) (void)hipEventDestroy(c->tev[j]);
      free_timing(c);
      return ffcv::check_hip(e, "ffcv_jpeg_set_timing: hipEventCreate");
    }
  }
  c->tev_cap = max_launches;
  c->tev_n = 0;
  return FFCV_OK;
}

int ffcv_jpeg_timing_read(ffcv_jpeg_ctx *c, float *ms, int max_launches, int *n_launches) {
  if (!c || !n_launches || (max_launches && !ms)) {
    ffcv::set_error("ffcv_jpeg_timing_read: invalid arguments");
    return FFCV_EINVAL;
  }
  const int n = c->tev_n < max_launches ? c->tev_n : max_launches;
  for (int i = 0; i < n; i++) {
    FFCV_HIP_CHECK(hipEventSynchronize(c->tev[4 * i + 3]));
    for (int q = 0; q < 3; q++) FFCV_HIP_CHECK(hipEventElapsedTime(&ms[3 * i + q], c->tev[4 * i + q], c->tev[4 * i + q + 1]));
  }
  *n_launches = n;
  c->tev_n = 0;
  return FFCV_OK;
}

// Diagnostic hook (not in the public header): the DC lane table the last
// RRC / FULL launch's entropy kernel wrote for images [0, n): lane_blk0[64]
// (first block each lane started, non-decreasing), lane_off[3][64] (the
// lanes' exclusive DC offsets per component) and the image status.
int ffcv_jpeg_lane_table(ffcv_jpeg_ctx *c, void *stream, int n, uint32_t *blk0, int32_t *off, int32_t *status) {
  if (!c || n < 0 || n > c->max_batch || !blk0 || !off || !status) {
    ffcv::set_error("ffcv_jpeg_lane_table: invalid arguments");
    return FFCV_EINVAL;
  }
  hipStream_t s = ffcv::as_stream(stream);
  ImgInfo *h = new ImgInfo[n > 0 ? n : 1];
  hipError_t e = hipMemcpyAsync(h, c->info, sizeof(ImgInfo) * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    delete[] h;
    return ffcv::check_hip(e, "ffcv_jpeg_lane_table");
  }
  for (int k = 0; k < n; k++) {
    status[k] = h[k].status;
    for (int l = 0; l < 64; l++) {
      blk0[64 * k + l] = h[k].lane_blk0[l];
      for (int q = 0; q < 3; q++) off[192 * k + 64 * q + l] = h[k].lane_off[q][l];
    }
  }
  delete[] h;
  return FFCV_OK;
}

// Diagnostic hook (not in the public header): the arena reservation the last
// launch's entropy kernel made for images [0, n) -- base offset and size in
// bytes (size 0: the image reserved nothing; K1 clears it for every image
// before the parse) -- and the arena's capacity.  Statuses come from the
// launch's own status array.
int ffcv_jpeg_arena_regions(ffcv_jpeg_ctx *c, void *stream, int n, uint64_t *base, uint64_t *size,
                            uint64_t *capacity) {
  if (!c || n < 0 || n > c->max_batch || !base || !size) {
    ffcv::set_error("ffcv_jpeg_arena_regions: invalid arguments");
    return FFCV_EINVAL;
  }
  hipStream_t s = ffcv::as_stream(stream);
  ImgInfo *h = new ImgInfo[n > 0 ? n : 1];
  hipError_t e = hipMemcpyAsync(h, c->info, sizeof(ImgInfo) * n, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    delete[] h;
    return ffcv::check_hip(e, "ffcv_jpeg_arena_regions");
  }
  for (int k = 0; k < n; k++) {
    base[k] = h[k].arena_base;
    size[k] = h[k].arena_need;
  }
  if (capacity) *capacity = c->arena_bytes;
  delete[] h;
  return FFCV_OK;
}

int ffcv_jpeg_set_entropy_index(ffcv_jpeg_ctx *c, uint32_t *index, uint64_t n_samples) {
  if (!c || (!index && n_samples)) {
    ffcv::set_error("ffcv_jpeg_set_entropy_index: invalid arguments");
    return FFCV_EINVAL;
  }
  c->eidx = index;
  c->eidx_n = index ? n_samples : 0;
  return FFCV_OK;
}

int ffcv_jpeg_arena_used(ffcv_jpeg_ctx *c, void *stream, uint64_t *used, uint64_t *capacity) {
  if (!c || !used) {
    ffcv::set_error("ffcv_jpeg_arena_used: invalid arguments");
    return FFCV_EINVAL;
  }
  unsigned long long v[2] = {0, 0};
  hipStream_t s = ffcv::as_stream(stream);
  FFCV_HIP_CHECK(hipMemcpyAsync(v, c->arena_top, sizeof(v), hipMemcpyDeviceToHost, s));
  FFCV_HIP_CHECK(hipStreamSynchronize(s));
  *used = c->arena_zero ? v[1] : v[0];
  if (capacity) *capacity = c->arena_bytes;
  return FFCV_OK;
}

int ffcv_jpeg_destroy(ffcv_jpeg_ctx *c) {
  if (c) free_ctx(c);
  return FFCV_OK;
}

static JpegArgs make_args(ffcv_jpeg_ctx *c, const uint8_t *base, const ffcv_sample *samples, int batch,
                          int32_t *status) {
  JpegArgs a = {};
  a.batch = batch;
  a.base = base;
  a.samples = samples;
  a.status = status;
  a.arena = c->arena;
  a.arena_bytes = c->arena_bytes;
  a.arena_top = c->arena_top;
  a.info = c->info;
  a.taps = c->taps;
  a.eidx = c->eidx;
  a.eidx_n = c->eidx_n;
  a.gtab = c->gtab;
  a.gtab_slot = c->gtab_slot;
  a.max_h = c->max_h;
  a.max_w = c->max_w;
  a.dbg = c->dbg;
  a.diag_only = c->diag_only;
  return a;
}

static int check_common(const char *fn, ffcv_jpeg_ctx *c, const uint8_t *base, const ffcv_sample *samples,
                        int batch, const void *out, const int32_t *status) {
  if (!c || !base || !samples || !out || !status || batch < 0) {
    ffcv::set_error("%s: invalid arguments", fn);
    return FFCV_EINVAL;
  }
  if (batch > c->max_batch) {
    ffcv::set_error("%s: batch %d exceeds ctx max_batch %d", fn, batch, c->max_batch);
    return FFCV_EINVAL;
  }
  return FFCV_OK;
}

// The bump counter must be 0 when K1 starts.  K2 zeroes it (its first
// workgroup, after K1 has finished on the stream), so a launch that follows
// one with K2 needs no memset: a memset is a kernel, and queued behind another
// stream's K1 it held this stream's K1 back by ~0.7 ms (rocprofv3 trace).
static int arena_before_k1(ffcv_jpeg_ctx *c, JpegArgs &a, hipStream_t s) {
  if (!c->arena_zero) FFCV_HIP_CHECK(hipMemsetAsync(a.arena_top, 0, sizeof(unsigned long long), s));
  c->arena_zero = false;
  return FFCV_OK;
}

static int launch_rrc(ffcv_jpeg_ctx *c, JpegArgs &a, hipStream_t s, const ffcv_rrc_params *p, void *out) {
  const int batch = a.batch;
  a.p = *p;
  a.out = out;
  const bool fp16 = p->lut != nullptr;
  uint64_t dense = (uint64_t)p->out_h * p->out_w * 3 * (fp16 ? 2 : 1);
  a.out_stride = p->out_stride ? p->out_stride : dense;
  const int only = a.diag_only;
  if (only & 1) {
    if (int rc = arena_before_k1(c, a, s)) return rc;
  }
  // per-kernel timing: events around each kernel on this stream
  hipEvent_t *ev = c->tev_n < c->tev_cap ? c->tev + 4 * c->tev_n++ : nullptr;
  if (ev) FFCV_HIP_CHECK(hipEventRecord(ev[0], s));
  if (only & 1) {
    if (c->k1_sorted && batch > JW * IPW) {
      hipLaunchKernelGGL(k1_order_kernel, dim3(1), dim3(K1O_T), 0, s, a, c->k1_order);
      FFCV_LAUNCH_CHECK("k1_order_kernel");
      a.k1_order = c->k1_order;
    }
    hipLaunchKernelGGL((jpeg_entropy_kernel<JM_RRC>), dim3((batch + JW * IPW - 1) / (JW * IPW)), dim3(JW * JT), K1_PAD,
                       s, a);
    a.k1_order = nullptr;
    FFCV_LAUNCH_CHECK("jpeg_entropy_kernel<RRC>");
  }
  if (ev) FFCV_HIP_CHECK(hipEventRecord(ev[1], s));
  if (only & 2) {
    hipLaunchKernelGGL(jpeg_idct_kernel, dim3(batch), dim3(K1B_T), 0, s, a);
    FFCV_LAUNCH_CHECK("jpeg_idct_kernel");
  }
  if (ev) FFCV_HIP_CHECK(hipEventRecord(ev[2], s));
  dim3 g2((p->out_h + BAND - 1) / BAND, batch);
  if (!(only & 4)) {
  } else if (fp16)
    hipLaunchKernelGGL((jpeg_color_resize_kernel<JM_RRC, true>), g2, dim3(K2T), K2_LDS, s, a);
  else
    hipLaunchKernelGGL((jpeg_color_resize_kernel<JM_RRC, false>), g2, dim3(K2T), K2_LDS, s, a);
  FFCV_LAUNCH_CHECK("jpeg_color_resize_kernel<RRC>");
  if (ev) FFCV_HIP_CHECK(hipEventRecord(ev[3], s));
  if (only & 4) c->arena_zero = true;
  return FFCV_OK;
}

int ffcv_jpeg_rrc_batch(ffcv_jpeg_ctx *c, void *stream, const uint8_t *base, const ffcv_sample *samples,
                        int batch, const int32_t *crops, const int32_t *cutout_yx, const uint8_t *flips,
                        const ffcv_rrc_params *p, void *out, int32_t *status) {
  int rc = check_common("ffcv_jpeg_rrc_batch", c, base, samples, batch, out, status);
  if (rc) return rc;
  if (!p || !crops || p->out_h <= 0 || p->out_w <= 0) {
    ffcv::set_error("ffcv_jpeg_rrc_batch: invalid params");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  JpegArgs a = make_args(c, base, samples, batch, status);
  a.crops = crops;
  a.cut = cutout_yx;
  a.flips = flips;
  return launch_rrc(c, a, ffcv::as_stream(stream), p, out);
}

int ffcv_jpeg_rrc_fused(ffcv_jpeg_ctx *c, void *stream, const uint8_t *base, const ffcv_sample *table,
                        uint64_t n_table, const uint64_t *ids, int batch, const ffcv_draw_params *dp,
                        int32_t *crops, int32_t *cutout_yx, uint8_t *flips, ffcv_sample *samples_out,
                        const ffcv_rrc_params *p, void *out, int32_t *status) {
  if (!c || !base || !table || !ids || !dp || !crops || !out || !status || batch < 0 || !p || p->out_h <= 0 ||
      p->out_w <= 0) {
    ffcv::set_error("ffcv_jpeg_rrc_fused: invalid arguments");
    return FFCV_EINVAL;
  }
  if (batch > c->max_batch) {
    ffcv::set_error("ffcv_jpeg_rrc_fused: batch %d exceeds ctx max_batch %d", batch, c->max_batch);
    return FFCV_EINVAL;
  }
  if (dp->out_h != p->out_h || dp->out_w != p->out_w || (cutout_yx && dp->cutout_size != p->cutout_size)) {
    ffcv::set_error("ffcv_jpeg_rrc_fused: draw and resize parameters disagree");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  JpegArgs a = make_args(c, base, nullptr, batch, status);
  a.table = table;
  a.n_table = n_table;
  a.ids = ids;
  a.samples_out = samples_out;
  a.dp = *dp;
  a.do_draw = 1;
  a.crops = a.crops_w = crops;
  a.cut = a.cut_w = cutout_yx;
  a.flips = a.flips_w = flips;
  return launch_rrc(c, a, ffcv::as_stream(stream), p, out);
}

int ffcv_jpeg_decode_batch(ffcv_jpeg_ctx *c, void *stream, const uint8_t *base, const ffcv_sample *samples,
                           int batch, uint8_t *out, uint64_t out_stride, int32_t *status) {
  int rc = check_common("ffcv_jpeg_decode_batch", c, base, samples, batch, out, status);
  if (rc) return rc;
  if (!out_stride) {
    ffcv::set_error("ffcv_jpeg_decode_batch: out_stride must be > 0");
    return FFCV_EINVAL;
  }
  if (batch == 0) return FFCV_OK;
  JpegArgs a = make_args(c, base, samples, batch, status);
  a.out = out;
  a.out_stride = out_stride;
  hipStream_t s = ffcv::as_stream(stream);
  if (int rc = arena_before_k1(c, a, s)) return rc;
  hipLaunchKernelGGL((jpeg_entropy_kernel<JM_FULL>), dim3((batch + JW * IPW - 1) / (JW * IPW)), dim3(JW * JT), 0, s, a);
  FFCV_LAUNCH_CHECK("jpeg_entropy_kernel<FULL>");
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3(batch), dim3(K1B_T), 0, s, a);
  FFCV_LAUNCH_CHECK("jpeg_idct_kernel");
  dim3 g2((c->max_h + BAND - 1) / BAND, batch);
  hipLaunchKernelGGL((jpeg_color_resize_kernel<JM_FULL, false>), g2, dim3(K2T), 0, s, a);
  FFCV_LAUNCH_CHECK("jpeg_color_resize_kernel<FULL>");
  c->arena_zero = true;
  return FFCV_OK;
}

int ffcv_jpeg_coefficients_batch(ffcv_jpeg_ctx *c, void *stream, const uint8_t *base,
                                 const ffcv_sample *samples, int batch, int16_t *coefs, uint64_t max_blocks,
                                 int32_t *status) {
  int rc = check_common("ffcv_jpeg_coefficients_batch", c, base, samples, batch, coefs, status);
  if (rc) return rc;
  if (batch == 0) return FFCV_OK;
  JpegArgs a = make_args(c, base, samples, batch, status);
  a.out = coefs;
  a.out_stride = max_blocks * 64 * 2;
  a.max_blocks = max_blocks;
  if (int rc2 = arena_before_k1(c, a, ffcv::as_stream(stream))) return rc2;
  hipLaunchKernelGGL((jpeg_entropy_kernel<JM_COEF>), dim3((batch + JW * IPW - 1) / (JW * IPW)), dim3(JW * JT), 0,
                     ffcv::as_stream(stream), a);
  FFCV_LAUNCH_CHECK("jpeg_entropy_kernel<COEF>");
  return FFCV_OK;
}

}  // extern "C"
