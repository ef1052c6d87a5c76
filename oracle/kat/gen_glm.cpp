// TEST INFRASTRUCTURE: golden-vector generator for camera / reprojection semantics.
// Compiled in the dev container against the reference's *vendored* glm 0.9.9 headers
// (/root/reference/template/src/pg/pg1_embree/glm, header-only).  The camera maths follows
// pg/camera.cpp:12-58,81-84 (Z-up, lookAt with recomputed up, pixel-corner primary rays) and
// the reprojection pg/ReSTIRIntegrator.cpp:544-565; every numeric operation is a genuine glm
// call, so the JSON (tests/golden/glm_kat.json) pins the restatement's matrix arithmetic.
#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>
#include <cstdio>
#include <cmath>

struct Cam { glm::vec3 from, at; float fov; int W, H; };

int main() {
    const Cam cams[] = {
        {{0.0f, -3.9f, 1.0f}, {0.0f, 0.0f, 1.0f}, 40.0f, 512, 512},
        {{1.878f, -7.724f, 1.602f}, {0.0f, 0.0f, 0.0f}, 55.0f, 1280, 720},
        {{0.3f, -3.5f, 1.2f}, {0.05f, 0.1f, 0.95f}, 40.0f, 1920, 1080},
        {{-2.5f, 1.5f, 3.0f}, {0.5f, -0.25f, 0.5f}, 66.0f, 640, 480},
    };
    const int pix[][2] = {{0, 0}, {1, 0}, {17, 33}, {100, 200}, {255, 255}, {300, 100}, {511, 511}, {639, 479}};
    const glm::vec3 pts[] = {{0.1f, 0.2f, 0.3f}, {-0.5f, 0.9f, 1.7f}, {0.0f, 0.0f, 0.0f}, {0.99f, -0.99f, 1.99f},
                             {0.3f, 2.0f, 0.5f}, {0.0f, 0.0f, 5.0f}};
    std::printf("{\n \"source\": \"glm 0.9.9 vendored at pg/pg1_embree/glm; pg/camera.cpp:12-84, pg/ReSTIRIntegrator.cpp:544-565\",\n");
    std::printf(" \"cameras\": [\n");
    for (int ci = 0; ci < 4; ++ci) {
        const Cam& c = cams[ci];
        float fov_y = glm::radians(c.fov);
        float f_y = static_cast<float>(c.H) / (2.0f * tanf(fov_y / 2.0f));
        const glm::vec3 up{0.0f, 0.0f, 1.0f};
        glm::vec3 z_c = glm::normalize(c.from - c.at);
        glm::vec3 x_c = glm::normalize(glm::cross(up, z_c));
        glm::vec3 y_c = glm::normalize(glm::cross(z_c, x_c));
        glm::mat4 view = glm::lookAt(c.from, c.at, y_c);
        glm::mat4 inv = glm::inverse(view);
        glm::mat3 invDir = glm::mat3(inv);
        std::printf("%s  {\"cam\": [%.9g, %.9g, %.9g, %.9g, %.9g, %.9g, %.9g], \"W\": %d, \"H\": %d,\n",
                    ci ? ",\n" : "", c.from.x, c.from.y, c.from.z, c.at.x, c.at.y, c.at.z, c.fov, c.W, c.H);
        std::printf("   \"focal\": %.9g,\n   \"view\": [", f_y);
        for (int k = 0; k < 16; ++k) std::printf("%s%.9g", k ? ", " : "", view[k / 4][k % 4]);
        std::printf("],\n   \"inv_view\": [");
        for (int k = 0; k < 16; ++k) std::printf("%s%.9g", k ? ", " : "", inv[k / 4][k % 4]);
        std::printf("],\n   \"rays\": [");
        bool first = true;
        for (auto& p : pix) {
            if (p[0] >= c.W || p[1] >= c.H) continue;
            glm::vec2 org{static_cast<float>(p[0]), static_cast<float>(p[1])};
            glm::vec3 d_c{org.x - static_cast<float>(c.W) / 2.0f, static_cast<float>(c.H) / 2.0f - org.y, -f_y};
            glm::vec3 d_w = glm::normalize(invDir * d_c);
            std::printf("%s[%d, %d, %.9g, %.9g, %.9g]", first ? "" : ", ", p[0], p[1], d_w.x, d_w.y, d_w.z);
            first = false;
        }
        std::printf("],\n   \"reproject\": [");
        first = true;
        for (auto& wp : pts) {
            glm::vec4 vh = view * glm::vec4(wp, 1.0f);
            glm::vec3 vs = glm::vec3(vh);
            int sx = -1, sy = -1;
            if (!(vs.z >= 0)) {
                int X = glm::round((-vs.x / vs.z) * f_y + static_cast<float>(c.W) / 2.0f);
                int Y = glm::round((vs.y / vs.z) * f_y + static_cast<float>(c.H) / 2.0f);
                if (!(X < 0 || X > c.W - 1 || Y < 0 || Y > c.H - 1)) { sx = X; sy = Y; }
            }
            std::printf("%s[%.9g, %.9g, %.9g, %d, %d]", first ? "" : ", ", wp.x, wp.y, wp.z, sx, sy);
            first = false;
        }
        std::printf("]}");
    }
    std::printf("\n ],\n \"disk_trunc\": [");
    // sampleDiskUniform result converted to glm::vec<2,int> (pg/ReSTIRIntegrator.cpp:338)
    const float offs[][2] = {{0.7f, -0.7f}, {-1.9f, 2.99f}, {5.477f, -5.477f}, {-0.0001f, 0.99999f}};
    for (int i = 0; i < 4; ++i) {
        glm::vec<2, int> o = glm::vec2{offs[i][0], offs[i][1]};
        std::printf("%s[%.9g, %.9g, %d, %d]", i ? ", " : "", offs[i][0], offs[i][1], o.x, o.y);
    }
    std::printf("],\n \"reflect\": [");
    const glm::vec3 I0 = glm::normalize(glm::vec3{0.3f, -0.8f, -0.52f});
    const glm::vec3 N0 = glm::normalize(glm::vec3{0.1f, 0.05f, 0.99f});
    glm::vec3 r = glm::normalize(glm::reflect(I0, N0));
    std::printf("%.9g, %.9g, %.9g, %.9g, %.9g, %.9g, %.9g, %.9g, %.9g]\n}\n", I0.x, I0.y, I0.z, N0.x, N0.y, N0.z, r.x, r.y, r.z);
    return 0;
}
