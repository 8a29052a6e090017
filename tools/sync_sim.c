// sync_sim.c -- host model of jpeg_entropy_kernel's parallel Huffman sync
// (P3), used to evaluate lane range sizes and guess heuristics without a GPU.
//   gcc -O2 -o /tmp/sync_sim tools/sync_sim.c && /tmp/sync_sim file.jpg [lanes] [heur]
// Prints rounds, the per-round maximum of symbols decoded by a lane (the
// latency proxy: rounds end at a workgroup barrier) and the total work.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int maxcode[18], valoff[17];
  uint8_t vals[256];
  uint16_t lut[1024];
  int ok;
} Huff;

static Huff H[8];
static int bpm, ph_dc[10], ph_ac[10];
static uint8_t *st;
static uint32_t dlen, tbits;

static uint32_t peek32(uint32_t pos) {
  uint64_t v = 0;
  uint32_t b = pos >> 3;
  for (int i = 0; i < 8; i++) v = (v << 8) | (b + i < dlen ? st[b + i] : 0);
  return (uint32_t)(v >> (32 - (pos & 7)));
}

// returns symbol, sets *len; *bad if no code
static int sym(int ti, uint32_t pos, int *len, int *bad) {
  uint32_t look = peek32(pos) >> 16;
  uint16_t e = H[ti].lut[look >> 6];
  *bad = 0;
  if (e >> 8) {
    *len = e >> 8;
    return e & 255;
  }
  for (int l = 11; l <= 16; l++) {
    int code = look >> (16 - l);
    if (code <= H[ti].maxcode[l]) {
      *len = l;
      return H[ti].vals[(H[ti].valoff[l] + code) & 255];
    }
  }
  *len = 16;
  *bad = 1;
  return 0;
}

typedef struct {
  uint32_t pos;
  int z, ph;
} St;

#define MAXEV 4096
typedef struct {
  uint32_t ev[MAXEV];
  uint32_t idx[MAXEV];  // blocks started before event q in this trajectory
  int nev;
  uint32_t cnt;  // blocks started from ev[0] on (or all if no drop)
  St exit;
} Traj;

static int heur = 0;
static long steps;

static uint32_t rec_from = 0;  // events / counts only at positions >= rec_from
// SIM_NEV: events kept per trajectory (0 = all); SIM_SPARSE=1: the kept
// events are the first block starts at or after NEV checkpoints spread over
// the lane range [rng_lo, end) instead of the first NEV block starts
static int nev_max = 0, sparse = 0;
static uint32_t rng_lo = 0;
static St run(St s, uint32_t end, Traj *t, const Traj *old, int spec) {
  int z = s.z, ph = s.ph;
  uint32_t pos = s.pos;
  uint32_t started = 0;
  int n = 0, j = 0, ck = 0;
  const int cap = nev_max ? nev_max : MAXEV;
  static Traj nt;
  nt.nev = 0;
  while (pos < end) {
    if (z == 0) {
      uint32_t key = (pos << 4) | ph;
      if (old) {
        while (j < old->nev && old->ev[j] < key) j++;
        if (j < old->nev && old->ev[j] == key) {
          for (int q = j; q < old->nev && n < cap; q++) {
            nt.ev[n] = old->ev[q];
            nt.idx[n++] = started + old->idx[q] - old->idx[j];
          }
          nt.nev = n;
          nt.cnt = started + old->cnt - old->idx[j];
          nt.exit = old->exit;
          *t = nt;
          return nt.exit;
        }
      }
      if (pos >= rec_from) {
        int rec = n < cap;
        if (sparse && nev_max) {
          uint32_t ckpos = rng_lo + (uint32_t)((uint64_t)(end - rng_lo) * ck / nev_max);
          rec = ck < nev_max && pos >= ckpos;
          if (rec) {
            while (ck < nev_max && pos >= rng_lo + (uint32_t)((uint64_t)(end - rng_lo) * ck / nev_max)) ck++;
          }
        }
        if (rec && n < MAXEV) {
          nt.ev[n] = key;
          nt.idx[n++] = started;
        }
        started++;
      }
    }
    steps++;
    int len, bad;
    int ti = z == 0 ? ph_dc[ph] : ph_ac[ph];
    int v = sym(ti, pos, &len, &bad);
    int sz = z == 0 ? v : (v & 15), r = z == 0 ? 0 : v >> 4;
    if (spec && heur) {
      int inval = bad || (z == 0 ? sz > 11 : (sz > 10 || (sz && z + r > 63) || (!sz && r == 15 && z + 16 > 63)));
      if (inval) {
        pos += len;
        z = 0;
        ph = (ph + 1) % bpm;
        n = 0;
        started = 0;
        continue;
      }
    }
    pos += len + sz;
    int zac = sz ? z + r + 1 : (r == 15 ? z + 16 : 64);
    z = z == 0 ? 1 : zac;
    if (z >= 64) {
      z = 0;
      ph = (ph + 1) % bpm;
    }
  }
  nt.nev = n;
  nt.cnt = started;
  nt.exit.pos = pos;
  nt.exit.z = z;
  nt.exit.ph = ph;
  *t = nt;
  return nt.exit;
}

static void build_huff(Huff *h, const uint8_t *cnt, const uint8_t *vals) {
  int code = 0, k = 0;
  for (int l = 1; l <= 16; l++) {
    if (cnt[l - 1]) {
      h->valoff[l] = k - code;
      code += cnt[l - 1];
      k += cnt[l - 1];
      h->maxcode[l] = code - 1;
    } else {
      h->maxcode[l] = -1;
      h->valoff[l] = 0;
    }
    code <<= 1;
  }
  memcpy(h->vals, vals, k);
  for (int v = 0; v < 1024; v++) {
    h->lut[v] = 0;
    for (int l = 1; l <= 10; l++) {
      int c = v >> (10 - l);
      if (c <= h->maxcode[l]) {
        h->lut[v] = (l << 8) | h->vals[(h->valoff[l] + c) & 255];
        break;
      }
    }
  }
  h->ok = 1;
}

int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "rb");
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *d = malloc(n);
  fread(d, 1, n, f);
  fclose(f);
  int lanes = argc > 2 ? atoi(argv[2]) : 256;
  heur = argc > 3 ? atoi(argv[3]) : 0;
  if (getenv("SIM_NEV")) nev_max = atoi(getenv("SIM_NEV"));
  if (getenv("SIM_SPARSE")) sparse = atoi(getenv("SIM_SPARSE"));
  long p = 2;
  int hs[3], vs[3], cid[3], nc = 0, scan = 0;
  while (!scan) {
    while (d[p] == 0xFF) p++;
    int m = d[p++];
    int len = (d[p] << 8) | d[p + 1];
    uint8_t *s = d + p + 2;
    if (m == 0xC4) {
      int o = 0;
      while (o < len - 2) {
        int tc = s[o] >> 4, th = s[o] & 15, tot = 0;
        for (int l = 0; l < 16; l++) tot += s[o + 1 + l];
        build_huff(&H[tc * 4 + th], s + o + 1, s + o + 17);
        o += 17 + tot;
      }
    } else if (m == 0xC0) {
      nc = s[5];
      for (int c = 0; c < nc; c++) {
        cid[c] = s[6 + 3 * c];
        hs[c] = s[7 + 3 * c] >> 4;
        vs[c] = s[7 + 3 * c] & 15;
      }
    } else if (m == 0xDA) {
      int ns = s[0];
      bpm = 0;
      for (int i = 0; i < ns; i++) {
        int c = 0;
        for (int q = 0; q < nc; q++)
          if (cid[q] == s[1 + 2 * i]) c = q;
        int nb = nc == 1 ? 1 : hs[c] * vs[c];
        for (int b = 0; b < nb; b++) {
          ph_dc[bpm] = s[2 + 2 * i] >> 4;
          ph_ac[bpm] = 4 + (s[2 + 2 * i] & 15);
          bpm++;
        }
      }
      scan = 1;
    }
    p += len;
  }
  st = malloc(n);
  dlen = 0;
  for (long q = p; q < n; q++) {
    if (d[q] == 0xFF) {
      if (q + 1 < n && d[q + 1] == 0) {
        st[dlen++] = 0xFF;
        q++;
        continue;
      }
      break;
    }
    st[dlen++] = d[q];
  }
  tbits = dlen * 8;
  if (heur == 8) {  // multi-symbol lookup: steps along the true trajectory when one
                    // lookup of PB bits resolves every whole symbol (code + extra
                    // bits) inside it, up to MS symbols, never past a block end
    int PB = getenv("SIM_PAIRB") ? atoi(getenv("SIM_PAIRB")) : 11;
    int MS = getenv("SIM_MS") ? atoi(getenv("SIM_MS")) : 2;
    int DCP = getenv("SIM_PAIRDC") ? atoi(getenv("SIM_PAIRDC")) : 0;
    uint32_t pos = 0;
    int z = 0, ph = 0;
    long nsym = 0, nstep = 0;
    while (pos < tbits) {
      nstep++;
      uint32_t p0 = pos;
      int k = 0;
      for (;;) {
        int len, bad, ti = z == 0 ? ph_dc[ph] : ph_ac[ph];
        int v = sym(ti, pos, &len, &bad);
        int sz = z == 0 ? v : (v & 15), r = z == 0 ? 0 : v >> 4;
        int dc = z == 0;
        if (k > 0 && (pos + len + sz - p0 > (uint32_t)PB || (dc && !DCP))) break;
        pos += len + sz;
        nsym++;
        k++;
        int zac = sz ? z + r + 1 : (r == 15 ? z + 16 : 64);
        z = z == 0 ? 1 : zac;
        if (z >= 64) {
          z = 0;
          ph = (ph + 1) % bpm;
          break;
        }
        if (k >= MS || pos >= tbits) break;
        if (dc && !DCP) break;
      }
    }
    printf("symbols %ld steps %ld (%.3f steps/symbol) PB %d MS %d DCP %d\n", nsym, nstep, (double)nstep / nsym, PB, MS, DCP);
    return 0;
  }
  if (heur == 10) {  // phase-probe heuristic: pick the start phase with the fewest implausible
                     // symbols over the first M symbols, then measure its phase-sync distance
    int M = getenv("SIM_PROBE") ? atoi(getenv("SIM_PROBE")) : 40;
    int8_t *tph = malloc(tbits + 64);
    memset(tph, -1, tbits + 64);
    uint32_t pos = 0;
    int z = 0, ph = 0;
    while (pos < tbits) {
      if (z == 0) tph[pos] = ph;
      int len, bad, ti = z == 0 ? ph_dc[ph] : ph_ac[ph];
      int v = sym(ti, pos, &len, &bad);
      int sz = z == 0 ? v : (v & 15), r = z == 0 ? 0 : v >> 4;
      pos += len + sz;
      int zac = sz ? z + r + 1 : (r == 15 ? z + 16 : 64);
      z = z == 0 ? 1 : zac;
      if (z >= 64) { z = 0; ph = (ph + 1) % bpm; }
    }
    srand(1);
    long s0sum = 0, sbsum = 0, s0max = 0, sbmax = 0, n = 0, right = 0;
    for (int smp = 0; smp < 400; smp++) {
      uint32_t s0 = (uint32_t)(((double)rand() / RAND_MAX) * (tbits * 0.8));
      int bestg = 0; long bestscore = 1L << 40;
      for (int g = 0; g < bpm; g++) {
        uint32_t q = s0; int zz = 0, pp = g; long score = 0;
        for (int k = 0; k < M && q < tbits; k++) {
          int len, bad, ti = zz == 0 ? ph_dc[pp] : ph_ac[pp];
          int v = sym(ti, q, &len, &bad);
          int sz = zz == 0 ? v : (v & 15), r = zz == 0 ? 0 : v >> 4;
          int inval = bad || (zz == 0 ? sz > 11 : (sz > 10 || (sz && zz + r > 63)));
          score += inval ? 100 : 0;
          score += zz == 0 ? 0 : 0;
          q += len + sz;
          int zac = sz ? zz + r + 1 : (r == 15 ? zz + 16 : 64);
          if (zz && zac > 64) score += 100;
          zz = zz == 0 ? 1 : zac;
          if (zz >= 64) { zz = 0; pp = (pp + 1) % bpm; }
        }
        if (score < bestscore) { bestscore = score; bestg = g; }
      }
      long dist[2];
      for (int w = 0; w < 2; w++) {
        int g = w ? bestg : 0;
        uint32_t q = s0; int zz = 0, pp = g; long k = 0, ps = -1;
        while (q < tbits && k < 200000) {
          if (zz == 0 && tph[q] == pp) { ps = k; break; }
          int len, bad, ti = zz == 0 ? ph_dc[pp] : ph_ac[pp];
          int v = sym(ti, q, &len, &bad);
          int sz = zz == 0 ? v : (v & 15), r = zz == 0 ? 0 : v >> 4;
          q += len + sz; k++;
          int zac = sz ? zz + r + 1 : (r == 15 ? zz + 16 : 64);
          zz = zz == 0 ? 1 : zac;
          if (zz >= 64) { zz = 0; pp = (pp + 1) % bpm; }
        }
        dist[w] = ps < 0 ? k : ps;
      }
      s0sum += dist[0]; sbsum += dist[1]; n++;
      if (dist[0] > s0max) s0max = dist[0];
      if (dist[1] > sbmax) sbmax = dist[1];
      right += dist[1] < 40;
    }
    printf("probe M=%d: guess0 mean %.1f max %ld | probe mean %.1f max %ld | synced<40 %.2f\n", M,
           (double)s0sum / n, s0max, (double)sbsum / n, sbmax, (double)right / n);
    return 0;
  }
  if (heur == 9) {  // sync-distance statistics from random starts
    int8_t *tph = malloc(tbits + 64);
    memset(tph, -1, tbits + 64);
    uint32_t pos = 0;
    int z = 0, ph = 0;
    while (pos < tbits) {
      if (z == 0) tph[pos] = ph;
      int len, bad, ti = z == 0 ? ph_dc[ph] : ph_ac[ph];
      int v = sym(ti, pos, &len, &bad);
      int sz = z == 0 ? v : (v & 15), r = z == 0 ? 0 : v >> 4;
      pos += len + sz;
      int zac = sz ? z + r + 1 : (r == 15 ? z + 16 : 64);
      z = z == 0 ? 1 : zac;
      if (z >= 64) { z = 0; ph = (ph + 1) % bpm; }
    }
    {
      long hist[18] = {0}, nsym = 0, bstart = 0;
      uint32_t q = 0; int zz = 0, pp = 0;
      while (q < tbits) {
        if (zz == 0) bstart++;
        int len, bad, ti = zz == 0 ? ph_dc[pp] : ph_ac[pp];
        int v = sym(ti, q, &len, &bad);
        int sz = zz == 0 ? v : (v & 15), r = zz == 0 ? 0 : v >> 4;
        hist[len]++; nsym++;
        q += len + sz;
        int zac = sz ? zz + r + 1 : (r == 15 ? zz + 16 : 64);
        zz = zz == 0 ? 1 : zac;
        if (zz >= 64) { zz = 0; pp = (pp + 1) % bpm; }
      }
      printf("symbols %ld blocks %ld sym/block %.2f bits/sym %.2f | len>10 %.4f len>11 %.4f len>12 %.4f\n", nsym, bstart,
             (double)nsym / bstart, (double)tbits / nsym,
             (double)(hist[11]+hist[12]+hist[13]+hist[14]+hist[15]+hist[16]) / nsym,
             (double)(hist[12]+hist[13]+hist[14]+hist[15]+hist[16]) / nsym,
             (double)(hist[13]+hist[14]+hist[15]+hist[16]) / nsym);
    }
    srand(1);
    long bs_sum = 0, ps_sum = 0, ps_max = 0, best_sum = 0, nsamp = 0;
    for (int smp = 0; smp < 300; smp++) {
      uint32_t s0 = (uint32_t)(((double)rand() / RAND_MAX) * (tbits * 0.8));
      long best = 1 << 30;
      for (int g = 0; g < bpm; g++) {
        uint32_t q = s0; int zz = 0, pp = g; long k = 0, bs = -1, ps = -1;
        while (q < tbits && k < 200000) {
          if (zz == 0) {
            if (bs < 0 && tph[q] >= 0) bs = k;
            if (tph[q] == pp) { ps = k; break; }
          }
          int len, bad, ti = zz == 0 ? ph_dc[pp] : ph_ac[pp];
          int v = sym(ti, q, &len, &bad);
          int sz = zz == 0 ? v : (v & 15), r = zz == 0 ? 0 : v >> 4;
          q += len + sz; k++;
          int zac = sz ? zz + r + 1 : (r == 15 ? zz + 16 : 64);
          zz = zz == 0 ? 1 : zac;
          if (zz >= 64) { zz = 0; pp = (pp + 1) % bpm; }
        }
        if (ps < 0) ps = k;
        if (g == 0) { bs_sum += bs; ps_sum += ps; if (ps > ps_max) ps_max = ps; nsamp++; }
        if (ps < best) best = ps;
      }
      best_sum += best;
    }
    printf("bit-sync mean %.1f sym | phase-sync (guess 0) mean %.1f max %ld | best-of-%d mean %.1f\n",
           (double)bs_sum / nsamp, (double)ps_sum / nsamp, ps_max, bpm, (double)best_sum / nsamp);
    return 0;
  }
  if (heur == 11) {  // write-pass split: lane ranges vs pieces of the prefix up to the
                     // block that starts MCU row SIM_ROWF * rows, cut at converged states
                     // (lane starts + the first NEV block starts on the 2^sh grid)
    double rowf = getenv("SIM_ROWF") ? atof(getenv("SIM_ROWF")) : 0.85;
    int NEVS = 6;
    uint32_t *sympos = malloc(sizeof(uint32_t) * (tbits + 2));  // symbols started before bit b
    uint32_t *bstart = malloc(sizeof(uint32_t) * (tbits / 6 + 16));
    int *bz = malloc(sizeof(int) * (tbits + 2));
    long nb = 0, ns = 0;
    uint32_t pos = 0;
    int z = 0, ph = 0;
    for (uint32_t b = 0; b <= tbits; b++) { sympos[b] = 0; bz[b] = -1; }
    while (pos < tbits) {
      bz[pos] = z;
      if (z == 0) bstart[nb++] = pos;
      int len, bad, ti = z == 0 ? ph_dc[ph] : ph_ac[ph];
      int v = sym(ti, pos, &len, &bad);
      int sz = z == 0 ? v : (v & 15), r = z == 0 ? 0 : v >> 4;
      uint32_t np = pos + len + sz;
      for (uint32_t b = pos + 1; b <= np && b <= tbits; b++) sympos[b] = ns + 1;
      ns++;
      pos = np;
      int zac = sz ? z + r + 1 : (r == 15 ? z + 16 : 64);
      z = z == 0 ? 1 : zac;
      if (z >= 64) { z = 0; ph = (ph + 1) % bpm; }
    }
    for (uint32_t b = pos; b <= tbits; b++) sympos[b] = ns;
    uint32_t cbits = (tbits + lanes - 1) / lanes;
    // lane starts: first symbol boundary >= t * cbits; its first block start; events
    uint32_t *ls = malloc(sizeof(uint32_t) * (lanes + 1));
    long *lb = malloc(sizeof(long) * (lanes + 1));
    uint32_t cand[4096];
    long candb[4096];
    int nc = 0;
    long bi = 0;
    double evq = ((double)nb / lanes + NEVS) / NEVS;
    int sh = 0;
    while ((1 << sh) < (int)evq) sh++;
    for (int t = 0; t < lanes; t++) {
      uint32_t p0 = t * cbits;
      while (p0 < tbits && bz[p0] < 0) p0++;
      ls[t] = p0;
      while (bi < nb && bstart[bi] < p0) bi++;
      lb[t] = bi;  // first block started at or after the lane start
      cand[nc] = p0;
      candb[nc++] = bz[p0] == 0 ? bi : -1;
      uint32_t end = (t + 1) * cbits;
      for (int q = 0; q < NEVS; q++) {
        long bq = bi + ((long)q << sh);
        if (bq < nb && bstart[bq] < end && bstart[bq] > p0) { cand[nc] = bstart[bq]; candb[nc++] = bq; }
      }
    }
    long need = (long)(rowf * nb);
    uint32_t E = tbits;
    for (int c = 0; c < nc; c++)
      if (candb[c] >= need) { E = cand[c]; break; }
    long base_max = 0, new_max = 0;
    for (int t = 0; t < lanes; t++) {
      uint32_t a = t * cbits, b = t == lanes - 1 ? tbits : (t + 1) * cbits;
      long s = (long)sympos[b < tbits ? b : tbits] - sympos[a < tbits ? a : tbits];
      if (s > base_max) base_max = s;
    }
    uint32_t *pc = malloc(sizeof(uint32_t) * (lanes + 1));
    for (int i = 0; i < lanes; i++) {
      uint32_t tg = (uint32_t)((uint64_t)i * E / lanes);
      uint32_t c0 = E;
      for (int c = 0; c < nc; c++)
        if (cand[c] >= tg) { c0 = cand[c]; break; }
      pc[i] = c0 < E ? c0 : E;
    }
    pc[lanes] = E;
    for (int i = 0; i < lanes; i++) {
      long s = pc[i + 1] > pc[i] ? (long)sympos[pc[i + 1]] - sympos[pc[i]] : 0;
      if (s > new_max) new_max = s;
    }
    printf("blocks %ld symbols %ld sh %d | E/total %.3f | lane-range max symbols %ld | piece max %ld (%.3f)\n", nb, ns,
           sh, (double)E / tbits, base_max, new_max, (double)new_max / base_max);
    return 0;
  }
  uint32_t cb = (tbits + lanes - 1) / lanes;
  Traj *T = calloc(lanes, sizeof(Traj));
  St *g = calloc(lanes, sizeof(St));
  long maxs = 0, tot = 0, wave_iters = 0, wmax[64] = {0};
  int warm = argc > 4 ? atoi(argv[4]) : 0;
  for (int t = 0; t < lanes; t++) {
    g[t].pos = t * cb;
    steps = 0;
    St st0 = g[t];
    st0.pos = t * cb > (uint32_t)warm ? t * cb - warm : 0;
    rec_from = t * cb;
    rng_lo = t * cb;
    run(t == 0 ? g[t] : st0, t == lanes - 1 ? tbits : (t + 1) * cb, &T[t], NULL, t > 0);
    rec_from = 0;
    if (steps > maxs) maxs = steps;
    if (steps > wmax[t / 64]) wmax[t / 64] = steps;
    tot += steps;
  }
  for (int q = 0; q < (lanes + 63) / 64; q++) { wave_iters += wmax[q]; wmax[q] = 0; }
  printf("bits %u bpm %d lanes %d range %u | r1 max %ld tot %ld\n", tbits, bpm, lanes, cb, maxs, tot);
  long lat = maxs, work = tot;
  int rounds = 0;
  for (;;) {
    St *ng = calloc(lanes, sizeof(St));
    int any = 0;
    for (int t = 0; t < lanes; t++) {
      ng[t] = t ? T[t - 1].exit : g[t];
      if (ng[t].pos != g[t].pos || ng[t].z != g[t].z || ng[t].ph != g[t].ph) any = 1;
    }
    if (!any) break;
    rounds++;
    long rm = 0;
    Traj *NT = calloc(lanes, sizeof(Traj));
    for (int t = 0; t < lanes; t++) {
      NT[t] = T[t];
      int ch = ng[t].pos != g[t].pos || ng[t].z != g[t].z || ng[t].ph != g[t].ph;
      if (!ch) continue;
      uint32_t end = t == lanes - 1 ? tbits : (t + 1) * cb;
      steps = 0;
      if (ng[t].pos >= end) {
        NT[t].nev = 0;
        NT[t].cnt = 0;
        NT[t].exit = ng[t];
      } else {
        rng_lo = t * cb;
        run(ng[t], end, &NT[t], &T[t], 0);
      }
      if (steps > rm) rm = steps;
      if (steps > wmax[t / 64]) wmax[t / 64] = steps;
      work += steps;
      if (getenv("SIM_DUMP")) printf("TASK %d %d %ld\n", rounds, t, steps);
    }
    for (int q = 0; q < (lanes + 63) / 64; q++) { wave_iters += wmax[q]; wmax[q] = 0; }
    memcpy(g, ng, lanes * sizeof(St));
    free(ng);
    free(T);
    T = NT;
    lat += rm;
    printf("  round %d max %ld\n", rounds, rm);
  }
  printf("rounds %d latency %ld work %ld (single pass %ld) wave-iters/wave %.0f\n", rounds, lat, work, tot,
         (double)wave_iters / ((lanes + 63) / 64));
  return 0;
}
