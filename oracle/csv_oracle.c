/* csv_oracle.c — TEST INFRASTRUCTURE ONLY (the checker for the device CSV decoder).
 *
 * CPU restatement of the reference's ingest parse, record by record:
 *   ServiceTuple.fromString          java/org.main/ServiceTuple.java:89-104
 *     s.split(",")                   (java.lang.String.split: trailing empty fields removed)
 *     p.length < 2 -> null           (:93)
 *     Double.parseDouble(p[i])       (:97; any exception -> null, :101-103)
 *   .filter(Objects::nonNull)        java/org.main/FlinkSkyline.java:103
 *   Long.parseLong(point.id)         java/org.main/FlinkSkyline.java:276 (throws -> task failure)
 *
 * Double.parseDouble's accepted syntax is restated from the JDK 11 grammar
 * (FloatingDecimal.readJavaFormatString / the HexFloatingPointLiteral regex of
 * Double.valueOf's javadoc): trim() of chars <= ' ', optional sign, "NaN",
 * "Infinity", hex significand with a mandatory binary exponent, decimal with an
 * optional e/E exponent, one optional trailing f/F/d/D.  The numeric value of an
 * accepted string is glibc strtod's (correctly rounded, round-half-even), which is
 * what the JDK's FloatingDecimal computes for decimal and hex input since JDK 8.
 * The JVM itself cannot run here (no JDK): this restatement is pinned against
 * Python's float() (David Gay's correctly rounded conversion) on the decimal
 * strings both grammars accept, and against a hand table of JDK behaviour
 * (tests/test_cpu_csv.py).
 *
 * Record status codes (same as the device's, include/skyline_hip.h SKY_CSV_*):
 *   0 ok, 1 malformed (fromString returns null), 2 the id does not parse as a
 *   Java long (the reference job would fail), 3 wrong arity (values != dims).
 */
#include <ctype.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Java String.trim(): strip chars <= ' ' at both ends */
static void jtrim(const char **s, const char **e) {
    while (*s < *e && (unsigned char)**s <= ' ') (*s)++;
    while (*e > *s && (unsigned char)(*e)[-1] <= ' ') (*e)--;
}

static int is_hex(int c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }

/* Double.parseDouble on [s, e): returns 1 and *out on success, 0 on NumberFormatException */
int orc_java_parse_double(const char *s0, const char *e0, double *out) {
    const char *s = s0, *e = e0;
    jtrim(&s, &e);
    if (s == e) return 0;
    int neg = 0;
    const char *p = s;
    if (*p == '+' || *p == '-') { neg = *p == '-'; p++; }
    if (p == e) return 0;
    if (*p == 'N') {
        if (e - p == 3 && memcmp(p, "NaN", 3) == 0) { *out = NAN; return 1; }
        return 0;
    }
    if (*p == 'I') {
        if (e - p == 8 && memcmp(p, "Infinity", 8) == 0) { *out = neg ? -INFINITY : INFINITY; return 1; }
        return 0;
    }
    char buf[8192];
    if (e - s >= (long)sizeof(buf)) return 0;   /* not reached by the tests */
    if (*p == '0' && e - p > 1 && (p[1] == 'x' || p[1] == 'X')) {
        /* 0[xX] (H+ .? | H* . H+) [pP] [+-]? D+ [fFdD]? */
        const char *q = p + 2;
        int nint = 0, nfrac = 0;
        while (q < e && is_hex(*q)) { q++; nint++; }
        if (q < e && *q == '.') { q++; while (q < e && is_hex(*q)) { q++; nfrac++; } }
        if (nint + nfrac == 0) return 0;
        if (q == e || (*q != 'p' && *q != 'P')) return 0;
        q++;
        if (q < e && (*q == '+' || *q == '-')) q++;
        int nexp = 0;
        while (q < e && *q >= '0' && *q <= '9') { q++; nexp++; }
        if (nexp == 0) return 0;
        const char *end = q;
        if (q < e && (*q == 'f' || *q == 'F' || *q == 'd' || *q == 'D')) q++;
        if (q != e) return 0;
        memcpy(buf, s, end - s);
        buf[end - s] = 0;
        *out = strtod(buf, NULL);
        return 1;
    }
    /* decimal: D* (. D*)? with >= 1 digit, ([eE] [+-]? D+)?, [fFdD]? */
    const char *q = p;
    int nd = 0;
    while (q < e && *q >= '0' && *q <= '9') { q++; nd++; }
    if (q < e && *q == '.') { q++; while (q < e && *q >= '0' && *q <= '9') { q++; nd++; } }
    if (nd == 0) return 0;
    if (q < e && (*q == 'e' || *q == 'E')) {
        q++;
        if (q < e && (*q == '+' || *q == '-')) q++;
        int ne = 0;
        while (q < e && *q >= '0' && *q <= '9') { q++; ne++; }
        if (ne == 0) return 0;
    }
    const char *end = q;
    if (q < e && (*q == 'f' || *q == 'F' || *q == 'd' || *q == 'D')) q++;
    if (q != e) return 0;
    memcpy(buf, s, end - s);
    buf[end - s] = 0;
    *out = strtod(buf, NULL);   /* overflow -> +-HUGE_VAL (= inf), underflow -> +-0 / subnormal: as Java */
    return 1;
}

/* Long.parseLong (radix 10, ASCII digits): no trimming, optional sign, >= 1 digit, range-checked */
int orc_java_parse_long(const char *s, const char *e, int64_t *out) {
    if (s == e) return 0;
    int neg = 0;
    if (*s == '+' || *s == '-') { neg = *s == '-'; s++; }
    if (s == e) return 0;
    uint64_t lim = neg ? (uint64_t)INT64_MAX + 1u : (uint64_t)INT64_MAX, v = 0;
    for (; s < e; s++) {
        if (*s < '0' || *s > '9') return 0;
        uint64_t d = (uint64_t)(*s - '0');
        if (v > (lim - d) / 10u) return 0;
        v = v * 10u + d;
    }
    *out = neg ? (int64_t)(0u - v) : (int64_t)v;
    return 1;
}

/* one record [s, e) -> status, id, values[D] */
static int parse_record(const char *s, const char *e, int D, int64_t *id, double *vals) {
    /* String.split(","): fields between commas; trailing empty fields removed */
    const char *fs[4096], *fe[4096];
    int nf = 0;
    const char *a = s;
    for (const char *q = s;; q++) {
        if (q == e || *q == ',') {
            if (nf == 4096) return 1;
            fs[nf] = a; fe[nf] = q; nf++;
            a = q + 1;
            if (q == e) break;
        }
    }
    while (nf > 0 && fs[nf - 1] == fe[nf - 1]) nf--;
    if (nf < 2) return 1;                                 /* ServiceTuple.java:93 */
    for (int i = 1; i < nf; i++) {
        double v;
        if (!orc_java_parse_double(fs[i], fe[i], &v)) return 1;
        if (i - 1 < D) vals[i - 1] = v;
    }
    if (!orc_java_parse_long(fs[0], fe[0], id)) return 2;   /* FlinkSkyline.java:276 */
    if (nf - 1 != D) return 3;
    return 0;
}

/* Records are '\n'-terminated; a non-empty unterminated tail is one more record.
 * Writes status[r] for every record and ids/vals[r] (row r) for status 0 rows;
 * returns the number of records. */
int64_t orc_parse_csv(const char *text, int64_t nbytes, int D, int64_t *ids, double *vals, uint8_t *status,
                      int64_t cap) {
    int64_t r = 0;
    const char *s = text, *end = text + nbytes;
    while (s < end) {
        const char *e = memchr(s, '\n', end - s);
        if (!e) e = end;
        if (r < cap) {
            int64_t id = 0;
            double tmp[64];
            int st = parse_record(s, e, D, &id, tmp);
            status[r] = (uint8_t)st;
            if (st == 0) {
                ids[r] = id;
                memcpy(vals + r * D, tmp, sizeof(double) * D);
            }
        }
        r++;
        s = e + 1;
    }
    return r;
}
