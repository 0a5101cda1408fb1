#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static float C[10]; static int NC;
static float at2(float y, float x) {
    float ax = fabsf(x), ay = fabsf(y);
    float mx = (ax > ay) ? ax : ay, mn = (ax > ay) ? ay : ax;
    if (mx < 0x1p-126f) mx = 0x1p-126f;
    uint32_t mb; memcpy(&mb, &mx, 4); mb = 0x7EF311C3u - mb; float r0; memcpy(&r0, &mb, 4);
    float e = fmaf(-mx, r0, 1.0f); float e2 = fmaf(e, e, e); r0 = fmaf(r0, e2, r0);
    e = fmaf(-mx, r0, 1.0f); r0 = fmaf(r0, e, r0);
    float a = mn * r0, s = a * a, p = C[NC-1];
    for (int i = NC-2; i >= 0; --i) p = fmaf(p, s, C[i]);
    float r = a * p;
    if (ay > ax) r = 0x1.921fb6p+0f - r;
    if (x < 0.0f) r = 0x1.921fb6p+1f - r;
    return copysignf(r, y);
}
int main(int argc, char** argv) {
    NC = argc - 1;
    for (int i = 0; i < NC; ++i) C[i] = strtof(argv[i+1], 0);
    double mx = 0; uint64_t st = 88172645463325252ull;
    for (long i = 0; i < 20000000; ++i) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        double u1 = ((st >> 11) + 0.5) / 9007199254740992.0;
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        double u2 = ((st >> 11) + 0.5) / 9007199254740992.0;
        float y = (float)(sqrt(-2*log(u1))*cos(6.283185307179586*u2)), x = (float)(sqrt(-2*log(u1))*sin(6.283185307179586*u2));
        double er = fabs((double)at2(y, x) - atan2((double)y, (double)x));
        if (er > mx) mx = er;
    }
    /* dense in a on the first octant */
    double mxa = 0;
    for (long i = 1; i <= 4000000; ++i) { float y = (float)i / 4000000.0f; double er = fabs((double)at2(y, 1.0f) - atan2((double)y, 1.0)); if (er > mxa) mxa = er; }
    printf("max err random %.3e  dense-octant %.3e\n", mx, mxa);
    return 0;
}
