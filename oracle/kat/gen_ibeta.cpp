// TEST INFRASTRUCTURE: golden-vector generator for the Phong energy normalisation.
// Compiled in the dev container against the reference's *vendored* Boost 1.86 headers
// (/root/reference/template/src/libs/Boost, header-only; sole use in the reference:
// pg/MaterialPhong.cpp:246-248 -> boost::math::beta(a, b, x), non-normalised incomplete beta).
// Nothing from the reference is copied; the output JSON (tests/golden/ibeta_kat.json) is data.
//
// calc_I_M below is evaluated with the genuine Boost ibeta and the float std::lgamma/std::exp/
// std::pow calls the reference uses (pg/MaterialPhong.cpp:224-244), so it pins the restatement.
#include <boost/math/special_functions/beta.hpp>
#include <cmath>
#include <cstdio>
#include <algorithm>

static float ibeta_ref(float x, float a, float b) { return boost::math::beta(a, b, x); }
static float gamma_quot(float a, float b) { return std::exp(std::lgamma(a) - std::lgamma(b)); }
static float calc_I_M(float nDotV, float n) {
    const float two_pi = 6.28318530717958647692528676655900576f;
    const float root_pi = 1.772453850905516027f;
    float costerm = nDotV;
    float sinterm_sq = 1.0f - costerm * costerm;
    float halfn = 0.5f * n;
    float negterm = costerm;
    sinterm_sq = std::min(std::max(sinterm_sq, 0.0f), 1.0f);
    if (n >= 1e-18f) negterm *= halfn * ibeta_ref(sinterm_sq, halfn, 0.5f);
    return (two_pi * costerm + root_pi * gamma_quot(halfn + 0.5f, halfn + 1.0f) *
            (std::pow(sinterm_sq, halfn) - negterm)) / (n + 2.0f);
}

int main() {
    std::printf("{\n \"source\": \"boost::math::beta (Boost 1.86 vendored at libs/Boost), pg/MaterialPhong.cpp:224-248\",\n");
    std::printf(" \"ibeta\": [\n");
    const double xs[] = {0.0, 1e-6, 0.001, 0.05, 0.1, 0.25, 0.5, 0.6, 0.75, 0.9, 0.99, 0.999999, 1.0};
    const double as[] = {0.05, 0.5, 1.0, 2.0, 4.0, 8.0, 16.0, 32.0, 64.0, 250.0, 1000.0};
    const double bs[] = {0.5, 1.0, 2.5};
    bool first = true;
    for (double a : as) for (double b : bs) for (double x : xs) {
        double v = boost::math::beta(a, b, x);
        std::printf("%s  [%.17g, %.17g, %.17g, %.17g]", first ? "" : ",\n", x, a, b, v);
        first = false;
    }
    std::printf("\n ],\n \"calc_I_M\": [\n");
    const float cs[] = {1.0f, 0.999f, 0.98f, 0.9f, 0.75f, 0.5f, 0.3f, 0.1f, 0.01f, 0.0f};
    const float ns[] = {0.0f, 1e-3f, 0.5f, 1.0f, 2.0f, 5.0f, 10.0f, 32.0f, 64.0f, 100.0f, 128.0f, 500.0f, 1000.0f};
    first = true;
    for (float n : ns) for (float c : cs) {
        float v = calc_I_M(c, n);
        std::printf("%s  [%.9g, %.9g, %.9g]", first ? "" : ",\n", (double)c, (double)n, (double)v);
        first = false;
    }
    std::printf("\n ]\n}\n");
    return 0;
}
