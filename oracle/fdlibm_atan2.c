/*
 * oracle/fdlibm_atan2.c — TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * CPU restatement of fdlibm 5.3 `s_atan.c` / `e_atan2.c`, the algorithm behind
 * `java.lang.StrictMath.atan2`, to which `java.lang.Math.atan2` delegates in
 * JDK 11 (the reference is a Java 11 job: /root/reference/pom.xml:11-39).
 * The reference calls it in AnglePartitioner.getKey
 * (/root/reference/java/org.main/FlinkSkyline.java:850).
 *
 * Third-party dependency: the JDK's fdlibm is NOT under /root/reference and no
 * JDK exists in this container, so the restatement is pinned by (a) the hex
 * words fdlibm publishes next to each constant (checked by
 * tests/test_cpu_oracle.py::test_fdlibm_constants_match_published_hex) and (b)
 * bit-exact agreement with V8's independent fdlibm port on the committed vectors
 * (tests/test_cpu_oracle.py::test_fdlibm_atan2_vs_v8_golden).  Compile with -ffp-contract=off: Java never contracts.
 */
#include <stdint.h>
#include <string.h>
#include <math.h>

static inline int32_t hi_word(double x) { uint64_t u; memcpy(&u, &x, 8); return (int32_t)(u >> 32); }
static inline uint32_t lo_word(double x) { uint64_t u; memcpy(&u, &x, 8); return (uint32_t)u; }
static inline double flip_sign(double x) { uint64_t u; memcpy(&u, &x, 8); u ^= 0x8000000000000000ull; memcpy(&x, &u, 8); return x; }

static const double atan_hi[4] = {
    4.63647609000806093515e-01, /* atan(0.5)hi 0x3FDDAC67 0x0561BB4F */
    7.85398163397448278999e-01, /* atan(1.0)hi 0x3FE921FB 0x54442D18 */
    9.82793723247329054082e-01, /* atan(1.5)hi 0x3FEF730B 0xD281F69B */
    1.57079632679489655800e+00, /* atan(inf)hi 0x3FF921FB 0x54442D18 */
};
static const double atan_lo[4] = {
    2.26987774529616870924e-17, /* 0x3C7A2B7F 0x222F65E2 */
    3.06161699786838301793e-17, /* 0x3C81A626 0x33145C07 */
    1.39033110312309984516e-17, /* 0x3C700788 0x7AF0CBBD */
    6.12323399573676603587e-17, /* 0x3C91A626 0x33145C07 */
};
static const double aT[11] = {
     3.33333333333329318027e-01, /* 0x3FD55555 0x5555550D */
    -1.99999999998764832476e-01, /* 0xBFC99999 0x9998EBC4 */
     1.42857142725034663711e-01, /* 0x3FC24924 0x920083FF */
    -1.11111104054623557880e-01, /* 0xBFBC71C6 0xFE231671 */
     9.09088713343650656196e-02, /* 0x3FB745CD 0xC54C206E */
    -7.69187620504482999495e-02, /* 0xBFB3B0F2 0xAF749A6D */
     6.66107313738753120669e-02, /* 0x3FB10D66 0xA0D03D51 */
    -5.83357013379057348645e-02, /* 0xBFADDE2D 0x52DEFD9A */
     4.97687799461593236017e-02, /* 0x3FA97B4B 0x24760DEB */
    -3.65315727442169155270e-02, /* 0xBFA2B444 0x2C6A6C2F */
     1.62858201153657823623e-02, /* 0x3F90AD3A 0xE322DA11 */
};

/* exported so the tests can compare each literal with its published hex word */
const double *orc_fdlibm_table(int which) {
    return which == 0 ? atan_hi : which == 1 ? atan_lo : aT;
}

double orc_fdlibm_atan(double x) {
    const double one = 1.0, huge = 1.0e300;
    int32_t hx = hi_word(x), ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x44100000) {                      /* |x| >= 2^66 */
        if (ix > 0x7ff00000 || (ix == 0x7ff00000 && lo_word(x) != 0)) return x + x;  /* NaN */
        return hx > 0 ? atan_hi[3] + atan_lo[3] : -atan_hi[3] - atan_lo[3];
    }
    if (ix < 0x3fdc0000) {                       /* |x| < 0.4375 */
        if (ix < 0x3e200000) {                   /* |x| < 2^-29 */
            if (huge + x > one) return x;
        }
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000) {                   /* |x| < 1.1875 */
            if (ix < 0x3fe60000) { id = 0; x = (2.0 * x - one) / (2.0 + x); }
            else                 { id = 1; x = (x - one) / (x + one); }
        } else {
            if (ix < 0x40038000) { id = 2; x = (x - 1.5) / (one + 1.5 * x); }
            else                 { id = 3; x = -1.0 / x; }
        }
    }
    double z = x * x;
    double w = z * z;
    double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    z = atan_hi[id] - ((x * (s1 + s2) - atan_lo[id]) - x);
    return hx < 0 ? -z : z;
}

double orc_fdlibm_atan2(double y, double x) {
    const double tiny = 1.0e-300, zero = 0.0;
    const double pi_o_4 = 7.8539816339744827900E-01;  /* 0x3FE921FB 0x54442D18 */
    const double pi_o_2 = 1.5707963267948965580E+00;  /* 0x3FF921FB 0x54442D18 */
    const double pi     = 3.1415926535897931160E+00;  /* 0x400921FB 0x54442D18 */
    const double pi_lo  = 1.2246467991473531772E-16;  /* 0x3CA1A626 0x33145C07 */
    int32_t hx = hi_word(x), ix = hx & 0x7fffffff;
    uint32_t lx = lo_word(x);
    int32_t hy = hi_word(y), iy = hy & 0x7fffffff;
    uint32_t ly = lo_word(y);
    if (((uint32_t)ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u ||
        ((uint32_t)iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
        return x + y;                                        /* NaN */
    if (((hx - 0x3ff00000) | (int32_t)lx) == 0) return orc_fdlibm_atan(y);   /* x == 1.0 */
    int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);              /* 2*sign(x)+sign(y) */
    if ((iy | (int32_t)ly) == 0) {                            /* y == 0 */
        switch (m) {
            case 0: case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if ((ix | (int32_t)lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;   /* x == 0 */
    if (ix == 0x7ff00000) {                                   /* x is INF */
        if (iy == 0x7ff00000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0 * pi_o_4 + tiny;
                default: return -3.0 * pi_o_4 - tiny;
            }
        } else {
            switch (m) {
                case 0: return zero;
                case 1: return -zero;
                case 2: return pi + tiny;
                default: return -pi - tiny;
            }
        }
    }
    if (iy == 0x7ff00000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;   /* y is INF */
    int k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = pi_o_2 + 0.5 * pi_lo;                     /* |y/x| > 2^60 */
    else if (hx < 0 && k < -60) z = 0.0;                      /* |y|/x < -2^60 */
    else z = orc_fdlibm_atan(fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return flip_sign(z);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}
