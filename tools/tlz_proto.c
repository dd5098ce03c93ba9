// tools/tlz_proto.c -- CPU simulation of the TLZ encoder (csrc/deflate_kernels.hip, gz::tlz) used to
// choose its parameters: member / segment size, window, chain candidates (NC), frontier entries (F),
// DP segment (S) and sweeps (SW), the cost model (ENTROPY=1: -log2 frequencies; else Huffman lengths),
// minimum match (minl), unrolled DP lengths (UNR=k).  Exact DEFLATE bit counting, header included.
//   gcc -O2 -o /tmp/tlz_proto tools/tlz_proto.c -lm
//   ENTROPY=1 /tmp/tlz_proto M C W NC F S SW NTOK [prior] [minl] < ids.u8   (ids: one byte per value)
// KC ranks (6 clusters): 131072 2048 8192 16 3 8 3 -> 0.1149; gzip -9 on the same bytes 0.1174.
// GPU-faithful simulation of the planned token-LZ encoder:
// member of M tokens, chunks of C tokens, window W tokens, 3-gram chains with
// up to NC candidates, nearest 1-/2-gram, frontier <= F steps, segmented DP
// (thread segments of S positions, SW sweeps, lookahead beyond handled by the
// shared cost array from the previous sweep), adaptive model per chunk.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

static int dist_code(uint32_t d) { if (d <= 4u) return (int)d - 1; uint32_t m = d - 1u; int b = 31 - __builtin_clz(m); return 2 * b + (int)((m >> (b - 1)) & 1u); }
static int dext(int c) { return c < 4 ? 0 : (c >> 1) - 1; }
static int len_code(uint32_t l) { if (l == 258u) return 28; uint32_t m = l - 3u; if (m < 8u) return (int)m; int b = 31 - __builtin_clz(m); return 4 * (b - 1) + (int)((m >> (b - 2)) & 3u); }
static int lext(int c) { return (c < 8 || c == 28) ? 0 : (c >> 2) - 1; }
static void huff(const double* f0, int n, int maxlen, int* len) {
    double w[600]; int par[600], sym[300]; char dead[600]; double f[300];
    memcpy(f, f0, sizeof(double) * n);
    for (;;) {
        int m = 0;
        for (int s = 0; s < n; ++s) { len[s] = 0; if (f[s] > 0) { sym[m] = s; w[m] = f[s]; ++m; } }
        if (m == 0) break;
        if (m == 1) { len[sym[0]] = 1; break; }
        for (int i = 0; i < 2 * m; ++i) { dead[i] = 0; par[i] = -1; }
        int nodes = m;
        for (int it = 0; it < m - 1; ++it) {
            int a = -1, b = -1;
            for (int i = 0; i < nodes; ++i) { if (dead[i]) continue; if (a < 0 || w[i] < w[a]) { b = a; a = i; } else if (b < 0 || w[i] < w[b]) b = i; }
            w[nodes] = w[a] + w[b]; dead[a] = dead[b] = 1; par[a] = par[b] = nodes; ++nodes;
        }
        int deep = 0;
        for (int i = 0; i < m; ++i) { int d = 0; for (int j = i; par[j] >= 0; j = par[j]) ++d; len[sym[i]] = d; if (d > deep) deep = d; }
        if (deep <= maxlen) break;
        for (int s = 0; s < n; ++s) if (f[s] > 0) f[s] = floor(f[s] / 2) + 1;
    }
}
static int header_bits(const int* ll, const int* ld) {
    int nlit = 257, ndist = 1;
    for (int i = 0; i < 286; ++i) if (ll[i]) nlit = i + 1 > nlit ? i + 1 : nlit;
    for (int i = 0; i < 30; ++i) if (ld[i]) ndist = i + 1 > ndist ? i + 1 : ndist;
    int v[320], N = nlit + ndist;
    for (int i = 0; i < nlit; ++i) v[i] = ll[i];
    for (int i = 0; i < ndist; ++i) v[nlit + i] = ld[i];
    double cf[19] = {0}; int rs[400], re[400], nr = 0;
    for (int i = 0; i < N;) {
        int j = i; while (j < N && v[j] == v[i]) ++j;
        int left = j - i, cur = v[i];
        if (cur == 0) { while (left >= 11) { int r = left < 138 ? left : 138; rs[nr] = 18; re[nr++] = 7; left -= r; } if (left >= 3) { rs[nr] = 17; re[nr++] = 3; left = 0; } while (left > 0) { rs[nr] = 0; re[nr++] = 0; --left; } }
        else { rs[nr] = cur; re[nr++] = 0; --left; while (left >= 3) { int r = left < 6 ? left : 6; rs[nr] = 16; re[nr++] = 2; left -= r; } while (left > 0) { rs[nr] = cur; re[nr++] = 0; --left; } }
        i = j;
    }
    for (int i = 0; i < nr; ++i) cf[rs[i]]++;
    int lc[19]; huff(cf, 19, 7, lc);
    static const int ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    int ncl = 19; while (ncl > 4 && lc[ord[ncl - 1]] == 0) --ncl;
    int bits = 3 + 5 + 5 + 4 + 3 * ncl;
    for (int i = 0; i < nr; ++i) bits += lc[rs[i]] + re[i];
    return bits;
}
static uint32_t tokbits(int t) { float f = (float)t; uint32_t u; memcpy(&u, &f, 4); return u; }

#define MAXF 16
int main(int argc, char** argv) {
    int M = atoi(argv[1]), C = atoi(argv[2]), W = atoi(argv[3]), NC = atoi(argv[4]), F = atoi(argv[5]);
    int S = atoi(argv[6]), SW = atoi(argv[7]), ntot = atoi(argv[8]);
    int prior = argc > 9 ? atoi(argv[9]) : 0; int minl = argc > 10 ? atoi(argv[10]) : 1;
    uint8_t* t = malloc(ntot + 128);
    if (fread(t, 1, ntot, stdin) != (size_t)ntot) return 1;
    memset(t + ntot, 255, 128);
    // frontier per position
    int* fl = malloc(sizeof(int) * ntot * MAXF); int* fg = malloc(sizeof(int) * ntot * MAXF); int* fn = calloc(ntot, sizeof(int));
    long long fsz[MAXF + 1] = {0};
    for (int i = 0; i < ntot; ++i) {
        int m0 = (i / M) * M, m1 = m0 + M < ntot ? m0 + M : ntot;
        int lo = i - W; if (lo < m0) lo = m0;
        int lim = 64; if (lim > m1 - i) lim = m1 - i;
        int n = 0, best = 0;
        // nearest 1-gram, 2-gram
        if (minl <= 1) for (int j = i - 1; j >= lo; --j) if (t[j] == t[i]) { int L = 1; while (L < lim && t[j + L] == t[i + L]) ++L; if (L > best) { fl[i * MAXF + n] = L; fg[i * MAXF + n] = i - j; ++n; best = L; } break; }
        if (lim >= 2 && minl <= 2) for (int j = i - 1; j >= lo; --j) if (t[j] == t[i] && t[j + 1] == t[i + 1]) { int L = 2; while (L < lim && t[j + L] == t[i + L]) ++L; if (L > best) { fl[i * MAXF + n] = L; fg[i * MAXF + n] = i - j; ++n; best = L; } break; }
        int cand = 0;
        if (lim >= 3) for (int j = i - 1; j >= lo && cand < NC; --j) if (t[j] == t[i] && t[j + 1] == t[i + 1] && t[j + 2] == t[i + 2]) {
            ++cand; int L = 3; while (L < lim && t[j + L] == t[i + L]) ++L;
            if (L > best) { if (n < MAXF) { fl[i * MAXF + n] = L; fg[i * MAXF + n] = i - j; ++n; } best = L; if (L == lim) break; }
        }
        fsz[n]++;
        // truncate to F: keep the first F-1 and the last (longest)
        if (n > F) { fl[i * MAXF + F - 1] = fl[i * MAXF + n - 1]; fg[i * MAXF + F - 1] = fg[i * MAXF + n - 1]; n = F; }
        fn[i] = n;
    }
    fprintf(stderr, "frontier sizes:"); for (int k = 0; k <= 8; ++k) fprintf(stderr, " %lld", fsz[k]); fprintf(stderr, "\n");
    double* cost = malloc(sizeof(double) * (ntot + 128));
    int* dec_l = malloc(sizeof(int) * ntot); int* dec_g = malloc(sizeof(int) * ntot);
    long long total_bits = 0, nops = 0;
    for (int m0 = 0; m0 < ntot; m0 += M) {
        int m1 = m0 + M < ntot ? m0 + M : ntot;
        double hl[286] = {0}, hd[30] = {0};
        double cl[286], cd[30];
        for (int s = 0; s < 286; ++s) cl[s] = 8; for (int s = 0; s < 30; ++s) cd[s] = 5;
        if (prior) { // prior: literal bytes 8, len codes 3..6 tokens cheap
            for (int s = 0; s < 286; ++s) cl[s] = 12; cl[0] = 2; cl[256+1] = 6;
            for (int l = 1; l <= 16; ++l) cl[257 + len_code(4 * l)] = 2 + (l > 6 ? l - 6 : 0);
            for (int c = 0; c < 30; ++c) cd[c] = 4;
        }
        int p = m0;  // parse position (continues across chunks)
        for (int c0 = m0; c0 < m1; c0 += C) {
            int c1 = c0 + C < m1 ? c0 + C : m1;
            // DP over [c0, c1 + 64): cost-to-go; positions >= c1 get linear estimate
            double rate = 4.0;  // bits per token estimate beyond
            for (int i = c1; i < c1 + 128; ++i) cost[i - m0 < 0 ? 0 : i] = rate * (i - c1);
            // initial for segmented sweeps: linear
            for (int i = c0; i < c1; ++i) cost[i] = rate * (c1 - i);
            for (int sw = 0; sw < SW; ++sw) {
                double* nc = malloc(sizeof(double) * (c1 - c0));
                for (int s0 = c0; s0 < c1; s0 += S) {
                    int s1 = s0 + S < c1 ? s0 + S : c1;
                    double loc[4096 + 128];
                    // local backward: positions >= s1 use cost[] from previous sweep (or final beyond chunk)
                    for (int i = s1 - 1; i >= s0; --i) {
                        #define CG(j) ((j) >= s1 ? cost[j] : loc[(j) - s0])
                        uint32_t b = tokbits(t[i]); double lc = 0; for (int k = 0; k < 4; ++k) lc += cl[(b >> (8 * k)) & 255];
                        double best = lc + CG(i + 1); int bl = 0, bg = 0;
                        int prevL = 0;
                        for (int k = 0; k < fn[i]; ++k) {
                            int L = fl[i * MAXF + k], g = fg[i * MAXF + k];
                            int dc = dist_code(4u * g); double dcost = cd[dc] + dext(dc);
                            int unr = getenv("UNR") ? atoi(getenv("UNR")) : 99;
                            for (int l = prevL + 1; l <= L; ++l) {
                                if (i + l > m1) break;
                                if (l > unr && l != L) continue;
                                int lcd = len_code(4u * l);
                                double cc = cl[257 + lcd] + lext(lcd) + dcost + CG(i + l);
                                if (cc < best) { best = cc; bl = l; bg = g; }
                            }
                            prevL = L;
                        }
                        loc[i - s0] = best; dec_l[i] = bl; dec_g[i] = bg;
                    }
                    for (int i = s0; i < s1; ++i) nc[i - c0] = loc[i - s0];
                }
                for (int i = c0; i < c1; ++i) cost[i] = nc[i - c0];
                free(nc);
            }
            // forward parse from p within the chunk (p may be > c0 from previous chunk's match)
            double chl[286] = {0}, chd[30] = {0};
            while (p < c1) {
                int l = dec_l[p];
                ++nops;
                if (l == 0) { uint32_t b = tokbits(t[p]); for (int k = 0; k < 4; ++k) chl[(b >> (8 * k)) & 255]++; p += 1; }
                else { chl[257 + len_code(4u * l)]++; chd[dist_code(4u * dec_g[p])]++; p += l; }
            }
            for (int s = 0; s < 286; ++s) hl[s] += chl[s];
            for (int s = 0; s < 30; ++s) hd[s] += chd[s];
            // adaptive model: from all chunks so far
            int ll[286], ld[30];
            double hl2[286], hd2[30];
            for (int s = 0; s < 286; ++s) hl2[s] = hl[s]; for (int s = 0; s < 30; ++s) hd2[s] = hd[s];
            hl2[256] += 1;
            if (getenv("ENTROPY")) {
                double tl = 0, td = 0; for (int s = 0; s < 286; ++s) tl += hl2[s]; for (int s = 0; s < 30; ++s) td += hd2[s];
                for (int s = 0; s < 286; ++s) cl[s] = hl2[s] > 0 ? fmax(1.0, log2(tl / hl2[s])) : log2(tl + 1) + 2;
                for (int s = 0; s < 30; ++s) cd[s] = hd2[s] > 0 ? fmax(1.0, log2(td / hd2[s])) : log2(td + 1) + 2;
            } else {
            huff(hl2, 286, 15, ll); huff(hd2, 30, 15, ld);
            for (int s = 0; s < 286; ++s) cl[s] = ll[s] ? ll[s] : 14;
            for (int s = 0; s < 30; ++s) cd[s] = ld[s] ? ld[s] : 10;
            }
        }
        hl[256] = 1;
        int ll[286], ld[30];
        huff(hl, 286, 15, ll); huff(hd, 30, 15, ld);
        long long bits = header_bits(ll, ld);
        for (int s = 0; s < 286; ++s) bits += (long long)hl[s] * ll[s];
        for (int s = 257; s < 286; ++s) bits += (long long)hl[s] * lext(s - 257);
        for (int s = 0; s < 30; ++s) bits += (long long)hd[s] * (ld[s] + dext(s));
        bits = (bits + 7) / 8 * 8 + 8 * 26;
        total_bits += bits;
    }
    printf("ratio %.5f ops %lld\n", total_bits / 8.0 / (4.0 * ntot), nops);
    return 0;
}
