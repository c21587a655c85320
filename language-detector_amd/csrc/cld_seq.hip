// cld_seq.hip -- spans for the documents the parallel span builder cannot
// formulate per character (included by cld_long.hip, inside namespace lng).
//
// next_span() derives every byte's role in a span from per-character
// properties.  That holds when the document tiles into well-formed characters
// whose scanner and lowercaser behaviour is local (classify(), lower_char);
// it does not for malformed UTF-8 (a lead byte claiming bytes that are not
// continuations, stray continuation bytes), for the HTML pages the rewrite
// (cld_html.hip) leaves alone, for documents past the slot's 1 MB letter-stop
// bitmap, or for a table set whose lowercaser does not keep ' '.  Those
// documents still run in k_long, through the same Squeeze / Repeats / hit /
// chunk / DocTote stages as every other document (detect() in "careful" mode:
// character starts by sequential decode, cld_long.hip char_starts): only their
// spans come from here.  Lane 0 walks the page the way the reference's scanner
// consumes it -- ScanToLetterOrSpecial over gaps, then one unit at a time (a
// character of UTF8OneCharLen bytes, a tag, a stray '>', an entity) -- and the
// lowercaser then runs over the whole span (LowerScriptSpan), so the span text
// is the reference's byte for byte.  These documents are rare: every corpus of
// the benchmark runs without one (tests/test_gpu_zfullsize.py).
//
// ResultChunkVector mode also needs ScriptScanner::MapBack for every byte of
// the lowered span (omap): map2original_ (the scanner's) composed with
// map2uplow_ (the lowercaser's).  Both are OffsetMaps built left to right and
// read only once they are complete, so each is kept as a stream of finished
// ranges (RangeStream) that writes the MapBack value of every A' position the
// moment its range is final: no op list is stored.

// OffsetMap (offsetmap.cc:104-200, MapBack :428-452) as a stream of finished
// ranges.  The pending range absorbs ops the way the reference merges them --
// the same op extends it; a Delete(1) followed by Insert(1), or an Insert(1)
// followed by Delete(1), turns it into Copy(1) -- and any other op finishes
// it.  (The reference's byte coding -- 6-bit lengths, prefix bytes, adjacent
// copies merged up to 63 -- changes no MapBack value.)  A finished range goes
// to the sink as (op, length, its first A offset, its first A' offset); MapBack
// of an A' position inside a Copy is its twin, inside an Insert the A offset
// the insert sits at, and past the last range (A' end) + (A end).
enum { kRangeCopy = 1, kRangeInsert = 2, kRangeDelete = 3 };
template <class Sink>
struct RangeStream {
  Sink sink;
  int op = kRangeCopy, len = 0;                  // the pending range (Clear(): a zero-length copy)
  int a = 0, ap = 0;                             // where it starts, in A and in A'
  bool any = false;                              // a range was finished (diffs_ not empty)
  __device__ void finish() {
    if (len == 0) return;
    sink(op, len, a, ap);
    any = true;
    if (op != kRangeInsert) a += len;
    if (op != kRangeDelete) ap += len;
    len = 0;
  }
  __device__ void start(int o, int n) {
    finish();
    op = o;
    len = n;
  }
  __device__ void copy(int n) {
    if (n == 0) return;
    if (op == kRangeCopy) len += n;
    else start(kRangeCopy, n);
  }
  __device__ void insert(int n) {
    if (n == 0) return;
    if (op == kRangeInsert) len += n;
    else if (n == 1 && op == kRangeDelete && len == 1) op = kRangeCopy;
    else start(kRangeInsert, n);
  }
  __device__ void del(int n) {
    if (n == 0) return;
    if (op == kRangeDelete) len += n;
    else if (n == 1 && op == kRangeInsert && len == 1) op = kRangeCopy;
    else start(kRangeDelete, n);
  }
  // Reset() -> MaybeFlushAll(): one more Copy(1) off the end when a range is
  // pending or none was ever finished.  Afterwards a = the A end, ap = the A' end.
  __device__ void reset() {
    if (len > 0 || !any) {
      copy(1);
      finish();
    }
  }
};

// map2original_: MapBack of every span-text position, into om (page offsets).
struct SpanSink {
  uint32_t* om;
  int cap;
  __device__ void operator()(int op, int len, int a, int ap) {
    if (op == kRangeDelete) return;
    for (int k = 0; k < len && ap + k < cap; ++k) om[ap + k] = (uint32_t)(op == kRangeCopy ? a + k : a);
  }
};
// map2uplow_ composed with map2original_: a lowered position's span-text
// position u (this map's MapBack), then om[u] (or the end rule past it).
struct LowerSink {
  uint32_t* omap;
  int cap;
  const uint32_t* om;                            // SpanSink's values
  int a_end, ap_end;                             // map2original_'s A and A' ends
  __device__ uint32_t back1(int u) const { return u < ap_end ? om[u] : (uint32_t)(u - ap_end + a_end); }
  __device__ void operator()(int op, int len, int a, int ap) {
    if (op == kRangeDelete) return;
    for (int k = 0; k < len && ap + k < cap; ++k) omap[ap + k] = back1(op == kRangeCopy ? a + k : a);
  }
};

// The page a sequential document is scanned from: the document as given (an
// HTML page the original, not its rewrite), and the scanner's mode.
struct SeqDoc {
  const uint8_t* p;
  int len;
  bool plain;                                    // is_plain_text
};

// What the scanner takes at byte p of the page: the unit's raw length (tlen),
// the bytes it puts into the span (plen, written to dst), and its script.
//  * an '&' in HTML mode is an entity (EntityToBuffer, getonescriptspan.cc:
//    454-468): its decoded character, or, undecodable, one byte and nothing
//    put -- and then *sc keeps the script the scanner last saw (it is not
//    assigned there, :874-883, 928-932);
//  * a '<' or '>' in HTML mode: in a run of letters it ends the run without
//    being consumed (in_run: tlen 0, :864-871); elsewhere a tag is skipped
//    whole (ScanToPossibleLetter, :150-203) and a '>' is one byte; script 0;
//  * anything else is one character of UTF8OneCharLen bytes -- continuation
//    bytes or not -- whose script is GetUTF8LetterScriptNum of its bytes.
__device__ __forceinline__ void seq_unit(const DevTables& T, const DocView& d, int p, int lim, bool plain, bool in_run,
                                         uint8_t* dst, int& tlen, int& plen, int& sc) {
  const uint8_t c = d.at(p);
  if (!plain && (c == '<' || c == '>')) {
    tlen = in_run ? 0 : (c == '<' ? scan_to_possible_letter(d, p, lim - p) : 1);
    plen = 0;
    sc = 0;
    return;
  }
  if (!plain && c == '&') {
    uint8_t tmp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    entity_to_buffer(T, d, p, lim - p, tmp, &tlen, &plen);
    for (int k = 0; k < plen; ++k) dst[k] = tmp[k];
    if (plen > 0) sc = script_num(T, BufView{tmp}, 0);
    return;
  }
  tlen = plen = utf8_len(c);
  for (int k = 0; k < plen; ++k) dst[k] = d.at(p + k);
  sc = script_num(T, d, p);
}

// One span of the page from byte `next` on (GetOneScriptSpan, getonescriptspan.cc:
// 799-1027, then LowerScriptSpan, :1033-1054), by lane 0: the raw span text in
// S.lb[1], lowered into lb with 40 NULs after it (the reference leaves one;
// nothing past the first four is read).  Returns text_bytes (filled - 3: it
// can be < 1 when the lowercaser stops at a malformed character early);
// *status 1, or 0 when no letter is left.  omap (vec mode): the page offset of
// every lowered byte (ScriptScanner::MapBack), with S.lbd as the span-text
// map's scratch (vec mode keeps no span cache).
template <bool VEC>
__device__ __forceinline__ int seq_span(const DevTables& T, const SeqDoc& q, Slot& S, uint8_t* lb, int& next, int& ulscript,
                        int& status, uint32_t* omap, int lane) {
  int tb = 0, ul = 0, st = 0, nx = next;
  if (lane == 0) {
    const DocView d{q.p, q.len};
    const int common = (int)T.common, inherited = (int)T.inherited;
    int remaining = q.len - nx;                                          // byte_length_
    // the soft limit splits the last two fragments of a long remainder in half (:814-819)
    const int soft = (kMaxScriptBytes <= remaining && remaining < 2 * kMaxScriptBytes)
                         ? remaining / 2 : kMaxScriptBytes - kWithinScriptTail;
    uint32_t* om = reinterpret_cast<uint32_t*>(S.lbd);
    RangeStream<SpanSink> m1{SpanSink{om, kMaxScriptBuffer + 16}};
    if (VEC) m1.del(nx);                                                 // MapBack(0) = the span offset (:835-836)
    uint8_t* raw = S.lb[1];
    uint8_t tmp[8];
    raw[0] = ' ';
    // SkipToFrontOfSpan (:589-642): gaps, tags and non-letters up to a letter
    int skip = 0, sc = 0, tlen = 0, plen = 0;
    while (skip < remaining) {
      skip += scan_to_letter_or_special(T, d, nx + skip, remaining - skip);
      if (skip >= remaining) {
        skip = remaining;
        break;
      }
      seq_unit(T, d, nx + skip, q.len, q.plain, false, tmp, tlen, plen, sc);
      if (sc != 0) break;
      skip += tlen;
    }
    const int spanscript = sc;
    nx += skip;
    remaining -= skip;
    if (VEC) {
      if (skip != 1) { m1.del(skip); m1.insert(1); }
      else m1.copy(1);
    }
    if (remaining > 0) {
      st = 1;
      ul = spanscript;
      const int base = nx, bl = remaining;
      int take = 0, put = 1;
      sc = 0;                                                            // UNKNOWN_ULSCRIPT (:823)
      while (take < bl) {
        // a run of same-script letters (with the single-letter exception, :887-912)
        for (;;) {
          if (take >= bl) break;
          seq_unit(T, d, base + take, q.len, q.plain, true, raw + put, tlen, plen, sc);
          if (tlen == 0) break;                                          // a tag or '>' ends the run
          bool brk = false;
          if (sc != spanscript && sc != inherited) {
            if (sc == common) brk = true;
            else {
              const int sc2 = script_num(T, d, base + take + tlen);      // the next character, raw bytes
              brk = sc2 != common && sc2 != spanscript;
            }
          }
          if (brk) break;
          take += tlen;
          put += plen;
          if (VEC) {
            if (tlen == plen) m1.copy(tlen);
            else if (tlen < plen) { m1.copy(tlen); m1.insert(plen - tlen); }
            else { m1.copy(plen); m1.del(tlen - plen); }
          }
          if (put >= kMaxScriptBytes) break;                             // the buffer is full (:948-952)
        }
        // a run of non-letters, tags and undecodable entities (:956-993)
        while (take < bl) {
          tlen = scan_to_letter_or_special(T, d, base + take, bl - take);
          take += tlen;
          if (VEC) m1.del(tlen);
          if (take >= bl) break;
          seq_unit(T, d, base + take, q.len, q.plain, false, tmp, tlen, plen, sc);
          if (sc != 0) break;
          take += tlen;
          if (VEC) m1.del(tlen);
        }
        raw[put++] = ' ';
        if (VEC) m1.insert(1);
        if (sc != spanscript && sc != inherited) break;                  // a letter of another script
        if (put >= soft) break;
      }
      // back up to a character boundary; the map is left as it is (:998-1004)
      while (0 < take && take < bl && (d.at(base + take) & 0xC0) == 0x80) {
        --take;
        --put;
      }
      nx += take;
      raw[put] = ' ';
      raw[put + 1] = ' ';
      raw[put + 2] = ' ';
      raw[put + 3] = 0;
      if (VEC) {
        m1.insert(4);
        m1.reset();
      }
      // LowerScriptSpan over the text and three of its pads (:1033-1054)
      int filled;
      if (VEC) {
        RangeStream<LowerSink> m2{LowerSink{omap, kLB, om, m1.a, m1.ap}};
        filled = lower_replace_sm(T.lower, raw, put + 3, lb, kMaxScriptLowerBuffer, q.plain, &m2);
        m2.reset();
        for (int t = m2.ap; t < filled + 8 && t < kLB; ++t) omap[t] = m2.sink.back1(t - m2.ap + m2.a);
      } else {
        filled = lower_replace_sm(T.lower, raw, put + 3, lb, kMaxScriptLowerBuffer, q.plain);
      }
      for (int k = 0; k < 40; ++k) lb[filled + k] = 0;
      tb = filled - 3;
    } else if (VEC) {
      m1.reset();
    }
  }
  gsync();
  tb = ufl(tb);
  ulscript = ufl(ul);
  status = ufl(st);
  next = ufl(nx);
  return tb;
}
