// TEST INFRASTRUCTURE: golden-vector generator that compiles the reference's OWN header-only code
// (no stand-ins): pg/Reservoir.h (LightSample / Reservoir::addSample / hasSample / capConfidence,
// :6-59), pg/Distribution.h (CosineWeightedDistribution / CosineLobeDistribution sample + getPdf,
// :7-68), pg/GBufferElement.h (GBufferElement::isValidForReSTIR, GBuffer::setAt layout, :6-89) and
// the inline helpers of pg/utils.h (Utils::powerHeuristic / maxComponent, :53-63), the MIS weights
// ReSTIRIntegrator::m_area / m_brdf (pg/ReSTIRIntegrator.h:62-74) and CenterSampler
// (pg/PixelSampler.h:12-17), with the vendored
// glm 0.9.9 (and the vendored Embree 3 headers, declarations only: Ray.h names RTCRay).  Built from the files where they lie under /root/reference by oracle/kat/Makefile; the
// only reference include that does not resolve on a case-sensitive file system, "Utils.h" in
// Distribution.h, is a symlink to the reference's own utils.h (oracle/_build/refinc/Utils.h).
//
// Two out-of-line members of Utils are defined here because their translation unit (pg/utils.cpp)
// includes the MSVC precompiled header and cannot be compiled:
//   * Utils::getRandomValue(a, b) (pg/utils.cpp:199-202) replays a recorded U stream: a + (b - a) * U,
//     so a fixture records which draws a function consumed, in order;
//   * Utils::orthogonal (pg/utils.cpp:204-207), restated verbatim (one expression).
// Output: tests/golden/refheaders_kat.json (floats printed with 9 significant digits = exact binary32).
#include <cfloat>
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <cmath>
#include <random>
#include <vector>

#include <memory>
#include <string>
#include <embree3/rtcore.h>   // vendored Embree 3.13.5 header: Ray.h (included by Reservoir.h) names RTCRay
#include <FreeImage.h>        // vendored FreeImage header: Texture.h (via material.h) names BYTE
#include <imgui.h>            // vendored ImGui header: PixelSampler.h (via camera.h) names ImGui
#include "utils.h"
#include "Reservoir.h"
#include "Distribution.h"
#include "GBufferElement.h"
#include "PixelSampler.h"
#include "ReSTIRIntegrator.h"

// ReSTIRIntegrator's sample-count statics (defined in pg/ReSTIRIntegrator.cpp:13-35); each m_area /
// m_brdf case below sets them
int ReSTIRIntegrator::M_Area = 1;
int ReSTIRIntegrator::M_Brdf = 1;

static std::vector<float> g_stream;
static size_t g_pos = 0;
static size_t g_draws = 0;

float Utils::getRandomValue(float a, float b) {
    const float u = g_stream[g_pos++ % g_stream.size()];
    ++g_draws;
    return a + (b - a) * u;
}
glm::vec3 Utils::orthogonal(const glm::vec3& vec) {
    return glm::abs(vec.x) > glm::abs(vec.z) ? glm::vec3{vec.y, -vec.x, 0.0f} : glm::vec3{0.0f, vec.z, -vec.y};
}

// a float as JSON: non-finite values (an M_Area of 0 divides by zero) as the strings "inf", "-inf", "nan"
static void pf(const char* sep, float v) {
    if (std::isfinite(v)) std::printf("%s%.9g", sep, v);
    else std::printf("%s\"%s\"", sep, std::isnan(v) ? "nan" : (v > 0 ? "inf" : "-inf"));
}
static void replay(const std::vector<float>& u) { g_stream = u; g_pos = 0; g_draws = 0; }
static void pv(const char* sep, const glm::vec3& v) { std::printf("%s%.9g, %.9g, %.9g", sep, v.x, v.y, v.z); }

int main() {
    std::mt19937 gen(20241016);
    std::uniform_real_distribution<float> U01(0.0f, 1.0f);
    auto u01 = [&] { return U01(gen); };
    std::printf("{\n \"source\": \"pg/Reservoir.h, pg/Distribution.h, pg/GBufferElement.h, pg/utils.h (inline helpers) compiled with the vendored glm 0.9.9; U streams replayed through Utils::getRandomValue\",\n");

    // ---------------------------------------------------------------- Reservoir::addSample streams
    // Each case: a sequence of (w, confidence) updates with a replayed U stream.  Sample i carries
    // samplePoint.x = i so the winner is identified; w mixes exact zeros (the w==0 && w_sum==0
    // early return), tiny, ordinary and huge weights.
    std::printf(" \"reservoir\": [\n");
    for (int c = 0; c < 96; ++c) {
        const int n = 1 + (int)(u01() * 40.0f);
        std::vector<float> w(n);
        std::vector<int> conf(n);
        for (int i = 0; i < n; ++i) {
            const float r = u01();
            if (c < 8 && i < n / 2) w[i] = 0.0f;                   // leading zeros: no draw consumed
            else if (r < 0.25f) w[i] = 0.0f;
            else if (r < 0.35f) w[i] = u01() * 1e-30f;
            else if (r < 0.45f) w[i] = u01() * 1e20f;
            else w[i] = u01() * 5.0f;
            conf[i] = (int)(u01() * 3.0f);
        }
        std::vector<float> us(n + 1);
        for (auto& x : us) x = u01();
        replay(us);
        Reservoir R{};
        std::vector<int> taken;
        for (int i = 0; i < n; ++i) {
            LightSample s{};
            s.samplePoint = glm::vec3{(float)i, 0.5f, -0.5f};
            s.sampleNormal = glm::vec3{0.0f, 0.0f, 1.0f};
            s.L_i = glm::vec3{1.0f, 2.0f, 3.0f};
            if (R.addSample(s, w[i], conf[i])) taken.push_back(i);
        }
        const int draws = (int)g_draws;
        const int cap = 1 + (c % 25);
        const int conf_before = R.confidence;
        R.capConfidence(cap);
        const int chosen = R.bestSample.samplePoint.x == -FLT_MAX ? -1 : (int)R.bestSample.samplePoint.x;
        std::printf("%s  {\"w\": [", c ? ",\n" : "");
        for (int i = 0; i < n; ++i) std::printf("%s%.9g", i ? ", " : "", w[i]);
        std::printf("], \"conf\": [");
        for (int i = 0; i < n; ++i) std::printf("%s%d", i ? ", " : "", conf[i]);
        std::printf("], \"u\": [");
        for (size_t i = 0; i < us.size(); ++i) std::printf("%s%.9g", i ? ", " : "", us[i]);
        std::printf("], \"cap\": %d, \"w_sum\": %.9g, \"confidence\": %d, \"confidence_capped\": %d, \"chosen\": %d, "
                    "\"draws\": %d, \"has_sample\": %d, \"valid\": %d, \"taken\": [",
                    cap, R.w_sum, conf_before, R.confidence, chosen, draws, R.hasSample() ? 1 : 0,
                    R.bestSample.isValid() ? 1 : 0);
        for (size_t i = 0; i < taken.size(); ++i) std::printf("%s%d", i ? ", " : "", taken[i]);
        std::printf("]}");
    }
    std::printf("\n ],\n");

    // ---------------------------------------------------------------- LightSample::isValid
    std::printf(" \"light_sample_valid\": [");
    {
        const float M = -FLT_MAX;
        const glm::vec3 cases[][3] = {
            {{0, 0, 0}, {0, 0, 1}, {1, 1, 1}}, {{M, 0, 0}, {0, 0, 1}, {1, 1, 1}}, {{0, 0, 0}, {0, M, 1}, {1, 1, 1}},
            {{0, 0, 0}, {0, 0, 1}, {0, 0, 0}}, {{0, 0, 0}, {0, 0, 1}, {-1, 0, 0.5f}}, {{M, M, M}, {M, M, M}, {M, M, M}},
            {{1, 2, 3}, {0, 1, 0}, {0, 0, 1e-30f}},
        };
        int i = 0;
        for (auto& cs : cases) {
            LightSample s{};
            s.samplePoint = cs[0]; s.sampleNormal = cs[1]; s.L_i = cs[2];
            std::printf("%s[", i++ ? ", " : "");
            pv("", cs[0]); pv(", ", cs[1]); pv(", ", cs[2]);
            std::printf(", %d]", s.isValid() ? 1 : 0);
        }
    }
    std::printf("],\n");

    // ---------------------------------------------------------------- Distribution.h
    std::vector<glm::vec3> dirs = {{0, 0, 1}, {0, 0, -1}, {1, 0, 0}, {0, 1, 0}, {-1, 0, 0}, {0.6f, 0.0f, 0.8f},
                                   {0.8f, 0.0f, 0.6f}, {0.70710677f, 0.0f, 0.70710677f}};
    std::normal_distribution<float> N01(0.0f, 1.0f);
    while (dirs.size() < 48) dirs.push_back(glm::normalize(glm::vec3{N01(gen), N01(gen), N01(gen)}));
    std::printf(" \"cosine_weighted\": [\n");
    int k = 0;
    for (const auto& n : dirs)
        for (int j = 0; j < 4; ++j) {
            const float r1 = j == 0 ? 0.0f : u01(), r2 = j == 1 ? 0.99999994f : u01();
            replay({r1, r2});
            const glm::vec3 wi = CosineWeightedDistribution::sample(n);
            const float pdf = CosineWeightedDistribution::getPdf(n, wi);
            const glm::vec3 other = dirs[(k * 7 + 3) % dirs.size()];
            const float pdf_other = CosineWeightedDistribution::getPdf(n, other);
            std::printf("%s  [", k++ ? ",\n" : "");
            pv("", n);
            std::printf(", %.9g, %.9g", r1, r2);
            pv(", ", wi);
            std::printf(", %.9g", pdf);
            pv(", ", other);
            std::printf(", %.9g]", pdf_other);
        }
    std::printf("\n ],\n \"cosine_lobe\": [\n");
    const float gammas[] = {0.0f, 1.0f, 2.0f, 8.0f, 16.0f, 64.0f, 127.5f, 1000.0f};
    k = 0;
    for (const auto& wr : dirs)
        for (int j = 0; j < 3; ++j) {
            const float g = gammas[(k + j) % 8];
            const float r1 = u01(), r2 = j == 0 ? 0.0f : u01();
            replay({r1, r2});
            const glm::vec3 wi = CosineLobeDistribution::sample(wr, g);
            const float pdf = CosineLobeDistribution::getPdf(wi, wr, g);
            const glm::vec3 other = dirs[(k * 5 + 1) % dirs.size()];
            const float pdf_other = CosineLobeDistribution::getPdf(other, wr, g);
            std::printf("%s  [", k++ ? ",\n" : "");
            pv("", wr);
            std::printf(", %.9g, %.9g, %.9g", g, r1, r2);
            pv(", ", wi);
            std::printf(", %.9g", pdf);
            pv(", ", other);
            std::printf(", %.9g]", pdf_other);
        }
    std::printf("\n ],\n");

    // ---------------------------------------------------------------- utils.h inline helpers
    std::printf(" \"power_heuristic\": [");
    const float ph[][2] = {{1, 1}, {0.5f, 2}, {3, 0}, {1e-20f, 1e-20f}, {7.25f, 0.125f}, {1e19f, 3e18f}, {0.0f, 2.0f}};
    for (int i = 0; i < 7; ++i)
        std::printf("%s[%.9g, %.9g, %.9g]", i ? ", " : "", ph[i][0], ph[i][1], Utils::powerHeuristic(ph[i][0], ph[i][1]));
    std::printf("],\n \"max_component\": [");
    for (int i = 0; i < 8; ++i) {
        const glm::vec3 v{u01() - 0.5f, u01() - 0.5f, u01() - 0.5f};
        pv(i ? "], [" : "[", v);
        std::printf(", %.9g", Utils::maxComponent(v));
    }
    std::printf("]],\n");

    // ---------------------------------------------------------------- ReSTIRIntegrator::m_area / m_brdf
    std::printf(" \"mis_area_brdf\": [");
    {
        const int MA[] = {1, 32, 0, 4, 32, 1, 7};
        const int MB[] = {1, 1, 1, 0, 2, 3, 5};
        const float pv_[][2] = {{0.0f, 0.0f}, {1.0f, 0.0f}, {0.0f, 2.5f}, {0.37f, 1.9f}, {1e-30f, 3e-31f},
                                {12.5f, 0.001f}, {1e20f, 1e19f}, {0.5f, 0.5f}};
        int i = 0;
        for (int m = 0; m < 7; ++m)
            for (auto& q : pv_) {
                ReSTIRIntegrator::M_Area = MA[m];
                ReSTIRIntegrator::M_Brdf = MB[m];
                const float a = ReSTIRIntegrator::m_area(q[0], q[1]);
                const float b = ReSTIRIntegrator::m_brdf(q[1], q[0]);
                std::printf("%s[%d, %d, %.9g, %.9g", i++ ? ", " : "", MA[m], MB[m], q[0], q[1]);
                pf(", ", a);
                pf(", ", b);
                std::printf("]");
            }
    }
    std::printf("],\n");
    {
        CenterSampler cs;
        const glm::vec2 o = cs.takeSample();
        std::printf(" \"center_sampler\": [%.9g, %.9g],\n", o.x, o.y);
    }

    // ---------------------------------------------------------------- GBufferElement / GBuffer
    std::printf(" \"gbuffer\": {\"size\": [7, 5], \"set\": [");
    {
        GBuffer gb(glm::vec<2, int>{7, 5});
        const int coords[][2] = {{0, 0}, {6, 0}, {0, 4}, {3, 2}, {6, 4}};
        for (int i = 0; i < 5; ++i) {
            GBufferElement e{};
            e.worldSpacePos = glm::vec3{(float)i, 1.0f, 2.0f};
            e.emission = i == 2 ? glm::vec3{0.0f, 0.0f, 1.0f} : glm::vec3{0.0f};
            e.shininess = 10.0f + i;
            e.depth = 0.5f * i;
            e.materialType = (MaterialType)(1 + i % 2);
            gb.setAt(glm::vec<2, int>{coords[i][0], coords[i][1]}, e);
            std::printf("%s[%d, %d, %d, %d]", i ? ", " : "", coords[i][0], coords[i][1], i,
                        e.isValidForReSTIR() ? 1 : 0);
        }
        // where each element landed in the SoA arrays: index of worldSpacePos.x == i, plus the other arrays
        std::printf("], \"linear_index\": [");
        int first = 1;
        for (size_t j = 0; j < gb.wSpacePositionBuf.size(); ++j)
            if (gb.wSpacePositionBuf[j].y == 1.0f) {
                std::printf("%s[%d, %zu, %.9g, %.9g, %d]", first ? "" : ", ", (int)gb.wSpacePositionBuf[j].x, j,
                            gb.shininessBuf[j], gb.depthBuf[j], (int)gb.matTypeBuf[j]);
                first = 0;
            }
        std::printf("], \"sizeof_element\": %zu}\n", sizeof(GBufferElement));
    }
    std::printf("}\n");
    return 0;
}
