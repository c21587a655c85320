// cld_html.hip -- HTML documents (cld_detect_batch_ex with CLD_FLAG_HTML,
// is_plain_text = false) on the parallel kernels.
//
// In HTML mode the reference's span scanner (getonescriptspan.cc:592-1027)
// differs from plain text in three ways only, all local to the bytes it meets:
//   * a '<' it reaches starts a tag, skipped by ScanToPossibleLetter (:150-203,
//     503-541), and a tag ends a run as any non-letter does;
//   * a '&' it reaches is an entity (ReadEntity, :393-451): a decoded character
//     is copied into the span in its place, an undecodable '&' is dropped (one
//     byte consumed, nothing copied, the run goes on);
//   * the lowercaser takes the HTML half of its remap pairs (:755-762).
// Every '<' and '&' outside a skipped tag or entity is reached (the scanner
// stops at both), so one left-to-right pass per document -- k_html_rewrite,
// one wavefront per page -- rewrites the page into a plain document with the
// same spans: each tag becomes one space, each entity its decoded bytes, a
// dropped '&' nothing, and the page keeps its length (spaces after the text:
// trailing spaces add nothing to any span).  k_wave / k_long then score it as
// plain text.  Two details keep them exact:
//   * a script lookahead (the next character's script, :1009-1016) that lands
//     on an entity saw the raw '&' (script 0): the rewrite marks those
//     positions in hflag, and the span builders read script 0 there;
//   * the lowercaser's HTML half: a page holding a character whose HTML-mode
//     lowering differs (kCptHtmlLower; for 4-byte characters one flag for the
//     whole range, k_build_cpt4 -- the reference's tables set neither), a
//     malformed character, or more than kHtmlRewriteMax bytes is not
//     rewritten and is scanned by k_long's sequential span source (cld_seq.hip);
//   * the span soft limit reads the raw bytes left (:814-819); it splits
//     nothing below kMaxScriptBytes (40,928), and for longer pages the rewrite
//     also records each output byte's page offset (hpos, with hgap after
//     dropped '&'s), from which the span builders read it (cld_long.hip
//     next_span).
// A rewritten page that k_long hands on goes to its SEQ instantiation, which
// scans the original page in HTML mode.
//
// One wavefront per page, in three steps (the reference's own pass is
// sequential, but only its '<' / '&' stops carry state):
//   1. the page goes to LDS (up to kHtmlStage bytes; longer pages are read in
//      place); every '<' and '&' of it is a candidate; each
//      lane evaluates one '&' as if the scan reached it (ReadEntity: bytes
//      consumed, bytes decoded) into an LDS list (a segment of the page at a
//      time: whole 64-byte windows holding at most kHtmlCands candidates);
//   2. the scan's order decides which candidates it reaches: a candidate
//      inside an earlier reached tag or entity is skipped (a scalar walk over
//      the list, 64 candidates per register); a reached '<' is scanned there,
//      by the whole wave, 64 bytes per step (scan_tag_wave);
//   3. per 64-byte window, each byte's output (a text byte: itself; a reached
//      tag: one space; a reached entity: its decoded bytes; a dropped '&' or a
//      byte inside a reached tag / entity: nothing) is placed by a prefix sum.

namespace cld {

using wave::dpp_scan_incl;
using wave::excl_scan;
using wave::lanemask_lt;
using wave::OpMax;
using wave::rdl;
using wave::rdlu;
using wave::wshr1;
using wave::wsum;
using wave::wsync;

constexpr int kHtmlRewriteMax = 64 << 20;  // (lng::kStBigMax) larger pages stay HTML (cld_seq.hip)
// LDS per wave (the page stage + the candidate lists) sets the resident waves
// of this latency-bound kernel: an 8 KB stage and 1,024 candidates per
// segment left 1.5 waves/SIMD; 2 KB and 256 (5.4 KB per wave) give 8, and
// the rewrite of 100 K 16 KB pages takes 21.4 ms instead of 48.2
// (profiles/round5_html_lds_ab.txt; 1 KB / 128 measured the same).
#ifndef HTML_STAGE
#define HTML_STAGE 2048
#endif
#ifndef HTML_CANDS
#define HTML_CANDS 256
#endif
#ifndef HTML_WPB
#define HTML_WPB 4
#endif
constexpr int kHtmlStage = HTML_STAGE;  // pages up to this size are staged in LDS, larger ones read in place
constexpr int kHtmlCands = HTML_CANDS;  // '<' / '&' candidates per segment of a page (round 5: any number per page)
constexpr int kHtmlWPB = HTML_WPB;      // waves (pages) per workgroup

// The character b0 b1 b2 b3 (n bytes) is well formed and lowers the same way
// in HTML mode as in plain text: a property-table bit for 1-3 byte
// characters, one flag for the whole 4-byte range (k_build_cpt4; never set by
// the reference's tables, so pages with emoji and other 4-byte characters are
// rewritten like any other page).
__device__ __forceinline__ bool html_lower_same(const DevTables& T, uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3,
                                                int n) {
  if (n >= 2 && (b1 & 0xC0) != 0x80) return false;
  if (n >= 3 && (b2 & 0xC0) != 0x80) return false;
  if (n == 4) return (b3 & 0xC0) == 0x80 && (gld(T.cpt + lng::kCptSize) & 1) == 0;
  return (gld(T.cpt + wave::cpt_index(b0, b1, b2, n)) & lng::kCptHtmlLower) == 0;
}

// ScanToPossibleLetter (getonescriptspan.cc:150-203, 503-541) with the tag
// parser's transition function as two LDS tables built from tag_class /
// tag_next (cld_prims.hip) at block start: one lookup per byte and no
// branch per state, so lanes in different states do not serialise.
constexpr int kTagStates = 40, kTagClasses = TC_PL + 1;
struct TagTables {
  uint8_t cls[256];
  uint8_t next[kTagStates * kTagClasses];
};
// The scan by the whole wave (uniform arguments): the parser sits in one
// state over long stretches (inside a tag, a quoted value, a comment, a
// script or style block), so each step tests the next 64 bytes at once --
// the transition each would make from the current state -- and jumps to the
// first byte that changes the state.
__device__ __forceinline__ int scan_tag_wave(const TagTables& tt, const uint8_t* text, int start, int len, int lane) {
  int src = start, e = 0, st = 0;
  const int lim = start + len;
  bool brk = false;
  while (src < lim) {
    const int x = src + lane;
    const int ns = tt.next[st * kTagClasses + tt.cls[x < lim ? text[x] : 0]];
    const uint64_t chg = __ballot(x < lim && ns != st);
    if (!chg) {                                  // 64 bytes (or the rest) in this state
      e = st;
      src = src + 64 < lim ? src + 64 : lim;
      continue;
    }
    const int k = __builtin_ctzll(chg);
    e = rdl(ns, k);
    src += k + 1;
    if (e <= 1) {
      --src;
      brk = true;
      break;
    }
    st = e;
  }
  (void)brk;
  if (src >= lim) return len;
  if (e != 0 && e != 2) {
    int off = src - start - 1;
    while (0 < off && text[start + off] != '<') --off;
    return off + 1;
  }
  return src - start;
}

struct HtmlSmem {
  uint8_t text[kHtmlStage + 16];       // the page (up to kHtmlStage bytes)
  uint32_t pos[kHtmlCands];            // candidate positions, in page order
  uint32_t len[kHtmlCands];            // bytes the scan consumes there
  uint32_t dec[kHtmlCands];            // an entity's decoded bytes
  uint8_t meta[kHtmlCands];            // kind (0 tag, 1 entity, 2 dropped '&') | plen << 2 | bad << 5 | reached << 6
};

// A byte of the page: staged pages are NUL padded in LDS; larger ones are read
// in place and bounded here.
template <bool kStaged>
__device__ __forceinline__ uint32_t txt_at(const uint8_t* txt, int p, int L) {
  return kStaged || p < L ? txt[p] : 0u;
}

// One page (steps 1-3 above).  txt is the page in LDS (kStaged, up to
// kHtmlStage bytes) or in place in HBM (up to kHtmlRewriteMax bytes).
template <bool kStaged>
__device__ __forceinline__ void rewrite_page(const DevTables& T, const TagTables& tt, HtmlSmem& S,
                                             const uint8_t* txt, const int L, const uint64_t a, const int i,
                                             const uint8_t sp, uint8_t* __restrict__ special,
                                             uint8_t* __restrict__ hbuf, uint8_t* __restrict__ hflag,
                                             uint32_t* __restrict__ hpos, uint32_t* __restrict__ hgap,
                                             const int hpos_min, unsigned long long* __restrict__ prof, const uint64_t am0,
                                             const uint64_t am1, const int lane) {
  const DocView dv{txt, L};
  // The page in segments of whole 64-byte windows holding at most kHtmlCands
  // candidates each: steps 1-2 per segment (the scan's reach carried in
  // `cur`), then step 3 over the segment's windows (its carries below).  A
  // tag or entity reached in one segment may run into the next: `cur` skips
  // the candidates it covers there, `cover` the text bytes.
  uint8_t* o = hbuf + a;
  uint8_t* f = hflag + a;
  uint32_t* hp = hpos && L >= hpos_min ? hpos + a : nullptr;
  uint32_t* hg = hp ? hgap + a : nullptr;
  int q = 0, bad = 0, conts = 0, need = 0, novec = 0;
  int drop_run = 0;                                            // dropped '&'s ending the previous window
  uint32_t cover = 0;                                          // end of the last reached candidate so far
  uint32_t drop_prev = 0;                                      // the byte before this window was a dropped '&'
  int cur = 0;                                                 // the scan's position after the last reached one
  for (int P0 = 0; P0 < L;) {
    // 1a. the segment's candidates, in page order: whole windows while they fit
    int K = 0, P1 = P0;
    for (int w0 = P0; w0 < L; w0 += 64) {
      const int p = w0 + lane;
      const uint32_t c = p < L ? txt[p] : 0u;
      const bool cand = c == '<' || c == '&';
      const uint64_t m = __ballot(cand);
      if (K + __popcll(m) > kHtmlCands) break;                 // (a window holds at most 64)
      if (cand) S.pos[K + __popcll(m & lanemask_lt(lane))] = (uint32_t)p;
      K += __popcll(m);
      P1 = w0 + 64 < L ? w0 + 64 : L;
    }
    wsync();
    // 1b. each candidate as if the scan reached it
    for (int j = lane; j < K; j += 64) {
      const int p = S.pos[j];
      int ln = 1, kind = 0, plen = 0;
      bool bd = false;
      uint32_t dec = 0;
      if (txt[p] == '<') {
        ln = 0;                                                // (a reached tag is scanned in step 2)
      } else {
        uint8_t tmp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int tlen = 0;
        entity_to_buffer(T, dv, p, L - p, tmp, &tlen, &plen);
        if (plen > 0) {
          kind = 1;
          ln = tlen;
          dec = (uint32_t)tmp[0] | ((uint32_t)tmp[1] << 8) | ((uint32_t)tmp[2] << 16) | ((uint32_t)tmp[3] << 24);
          bd = !html_lower_same(T, tmp[0], tmp[1], tmp[2], tmp[3], plen) ||
               (tmp[0] < 0x80 && (((tmp[0] < 64 ? am0 : am1) >> (tmp[0] & 63)) & 1));
        } else {
          kind = 2;                                            // undecodable: the '&' is dropped
          plen = 0;
        }
      }
      S.len[j] = (uint32_t)ln;
      S.dec[j] = dec;
      S.meta[j] = (uint8_t)(kind | (plen << 2) | (bd ? 0x20 : 0));
    }
    wsync();
    // 2. which candidates the scan reaches: past the end of the last reached one
    const long long t2 = prof ? (long long)clock64() : 0;
    for (int j0 = 0; j0 < K; j0 += 64) {
      const int j = j0 + lane;
      const int p = j < K ? (int)S.pos[j] : 0x7FFFFFFF, ln = j < K ? (int)S.len[j] : 0;
      const int m = K - j0 < 64 ? K - j0 : 64;
      const uint64_t tag_m = __ballot(j < K && (S.meta[j] & 3) == 0);
      uint64_t reach = 0;
      for (int t = 0; t < m; ++t) {
        const int pt = rdl(p, t);
        if (pt >= cur) {
          reach |= 1ull << t;
          int lt = rdl(ln, t);
          if ((tag_m >> t) & 1) {                    // a reached tag: ScanToPossibleLetter, by the wave
            lt = scan_tag_wave(tt, txt, pt, L - pt, lane);
            if (lane == t) S.len[j] = (uint32_t)lt;
          }
          cur = pt + lt;
        }
      }
      if (j < K) S.meta[j] = (uint8_t)(S.meta[j] | (((reach >> lane) & 1) ? 0x40 : 0));
    }
    wsync();
    if (prof && lane == 0) atomicAdd(prof, (unsigned long long)((long long)clock64() - t2));
    // 3. the output, window by window
    int cb = 0;
    for (int w0 = P0; w0 < P1; w0 += 64) {
      const int p = w0 + lane;
      const bool in = p < L;
      const uint32_t c = in ? txt[p] : 0u;
      const bool cand = in && (c == '<' || c == '&');
      const uint64_t cm = __ballot(cand);
      const int j = cand ? cb + __popcll(cm & lanemask_lt(lane)) : 0;
      cb += __popcll(cm);
      const uint32_t meta = cand ? S.meta[j] : 0u;
      const bool reached = (meta & 0x40) != 0;
      const uint32_t end = reached ? (uint32_t)(p + S.len[j]) : 0u;
      // covered: inside a reached candidate that starts before p (the running
      // maximum of reached ends, carried across windows and segments)
      const uint32_t mx = dpp_scan_incl(end, 0u, OpMax());
      const uint32_t before = wshr1(mx, 0u);
      const uint32_t cov_end = before > cover ? before : cover;
      const bool covered = in && !reached && (uint32_t)p < cov_end;
      const int kind = meta & 3, plen = (meta >> 2) & 7;
      const bool text = in && !covered && !reached;
      int emit = 0;
      if (reached) emit = kind == 0 ? 1 : kind == 1 ? plen : 0;
      else if (text) emit = 1;
      // the first byte after a dropped '&' carries the lookahead mark
      const bool dropped = reached && kind == 2;
      const uint32_t dprev = wshr1(dropped ? 1u : 0u, drop_prev);
      const int at = q + excl_scan(emit, lane);
      // vec mode (hpos): every output byte's page offset, as map2original_ maps
      // it -- a text byte its own, a tag's space the tag start, an entity's k-th
      // byte start + k (Copy(plen), then Delete(tlen - plen)).  An entity whose
      // Delete is a single byte, or that grows (Insert), could merge with the
      // run's closing Insert(1) into a Copy (offsetmap.cc:122-156): such pages
      // keep the sequential span source in vec mode (kSpecialNoVec).
      // the first byte after dropped '&'s also records where they began (hpos
      // second half, read where hflag bit 1 is set): a run ending there has its
      // gap start at the first of them (they merge into the gap's Delete)
      const uint64_t dm = __ballot(dropped);
      if (hp && dprev) {
        const uint64_t nd = ~dm & lanemask_lt(lane);             // bytes before this one that were not dropped
        const int first = nd ? w0 + (63 - __builtin_clzll(nd)) + 1 : w0 - drop_run;
        hg[at] = (uint32_t)first;
      }
      drop_run = dm == ~0ull ? drop_run + 64 : (int)__builtin_clzll(~dm);   // dropped bytes ending the window
      if (hp) {
        if (text || (reached && kind == 0)) hp[at] = (uint32_t)p;
        if (reached && kind == 1) {
          for (int k = 0; k < plen; ++k) hp[at + k] = (uint32_t)(p + k);
          const int tl = S.len[j];
          if (tl - plen == 1 || plen > tl) novec = 1;
        }
      }
      if (text) {
        o[at] = (uint8_t)c;
        f[at] = (uint8_t)(dprev ? 3 : 0);          // bit 1: the byte after a dropped '&'

        // plain characters: well formed, and the same lowering in HTML mode
        if (c < 0x80) {
          bad |= (((c < 64 ? am0 : am1) >> (c & 63)) & 1) ? 1 : 0;
        } else if ((c & 0xC0) == 0x80) {
          ++conts;
        } else {
          const int mm = utf8_len((uint8_t)c);
          const uint32_t b1 = txt_at<kStaged>(txt, p + 1, L), b2 = txt_at<kStaged>(txt, p + 2, L),
                         b3 = mm == 4 ? txt_at<kStaged>(txt, p + 3, L) : 0u;
          bad |= (p + mm > L || !html_lower_same(T, c, b1, b2, b3, mm)) ? 1 : 0;
          need += mm - 1;
        }
      } else if (reached && kind == 0) {
        o[at] = ' ';
        f[at] = (uint8_t)(dprev ? 3 : 0);
      } else if (reached && kind == 1) {
        const uint32_t d = S.dec[j];
        for (int k = 0; k < plen; ++k) {
          o[at + k] = (uint8_t)(d >> (8 * k));
          f[at + k] = k == 0 ? 1 : 0;
        }
        bad |= (meta & 0x20) ? 1 : 0;
      }
      q = rdl(at + emit, 63);
      const uint32_t wmx = rdlu(mx, 63);
      cover = wmx > cover ? wmx : cover;
      drop_prev = rdlu(dropped ? 1u : 0u, 63);
    }
    wsync();                                                   // S.* reused by the next segment
    P0 = P1;
  }
  // the page keeps its length: spaces after the text
  for (int p = q + lane; p < L; p += 64) {
    o[p] = ' ';
    f[p] = 0;
    if (hp) hp[p] = (uint32_t)L;
  }
  bad |= wsum(conts - need) != 0 ? 1 : 0;                      // every continuation byte claimed
  const bool nv = __ballot(novec != 0) != 0;
  if (__ballot(bad != 0) == 0 && lane == 0)
    special[i] = (uint8_t)((sp & ~kSpecialHtml) | kSpecialRewritten | (nv ? kSpecialNoVec : 0));
}

__global__ __launch_bounds__(64 * kHtmlWPB) void k_html_rewrite(const DevTables* __restrict__ Tp,
                                                               const uint8_t* __restrict__ buf,
                                                               const uint64_t* __restrict__ offs, int n,
                                                               uint8_t* __restrict__ special,
                                                               uint8_t* __restrict__ hbuf, uint8_t* __restrict__ hflag,
                                                               uint32_t* __restrict__ hpos, uint32_t* __restrict__ hgap,
                                                               int hpos_min, unsigned long long* __restrict__ prof) {
  __shared__ HtmlSmem smem[kHtmlWPB];
  __shared__ TagTables tt;
  for (int t = threadIdx.x; t < 256 + kTagStates * kTagClasses; t += blockDim.x) {
    if (t < 256) tt.cls[t] = (uint8_t)tag_class((uint8_t)t);
    else tt.next[t - 256] = (uint8_t)tag_next((t - 256) / kTagClasses, (t - 256) % kTagClasses);
  }
  __syncthreads();
  const DevTables& T = *Tp;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  HtmlSmem& S = smem[wv];
  // ASCII characters whose HTML-mode lowering differs: a 128-bit mask
  const uint64_t am0 = __ballot((gld(T.cpt + lane) & lng::kCptHtmlLower) != 0);
  const uint64_t am1 = __ballot((gld(T.cpt + 64 + lane) & lng::kCptHtmlLower) != 0);
  const int nw = gridDim.x * kHtmlWPB;
  for (int i = blockIdx.x * kHtmlWPB + wv; i < n; i += nw) {
    const uint8_t sp = special[i];
    if (!(sp & kSpecialHtml)) continue;
    const uint64_t a = offs[i];
    const int64_t len64 = (int64_t)(offs[i + 1] - a);
    if (len64 > kHtmlRewriteMax) continue;                       // stays HTML: cld_seq.hip
    const int L = (int)len64;
    if (L > kHtmlStage) {
      rewrite_page<false>(T, tt, S, buf + a, L, a, i, sp, special, hbuf, hflag, hpos, hgap, hpos_min, prof, am0, am1,
                          lane);
    } else {
      // the page into LDS (from aligned dwords), NUL padded
      const uint8_t* g = buf + a;
      for (int p = lane * 4; p < L + 16; p += 256) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) v |= (uint32_t)(p + k < L ? g[p + k] : 0) << (8 * k);
        *reinterpret_cast<uint32_t*>(&S.text[p]) = v;
      }
      wsync();
      rewrite_page<true>(T, tt, S, S.text, L, a, i, sp, special, hbuf, hflag, hpos, hgap, hpos_min, prof, am0, am1,
                         lane);
    }
    wsync();
  }
}

}  // namespace cld
