// C++ scene-model checks (include/sr/scene.hpp), built against libsr.so and
// run by tests/test_cpp_scene.py. No GPU needed: only host code is exercised.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "sr/scene.hpp"

static int failures = 0;
#define CHECK(cond)                                                        \
    do {                                                                   \
        if (!(cond)) {                                                     \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);    \
            failures++;                                                    \
        }                                                                  \
    } while (0)

using namespace sr;

int main() {
    // ObjectLoader singleton + DefaultScene == sr_default_scene (minus texture sizes)
    {
        DefaultScene d;
        ObjectLoader* L = ObjectLoader::getInstance();
        CHECK(L == ObjectLoader::getInstance());
        L->clear();
        d.registerWith(*L);
        sr_scene a, b;
        sr_scene_clear(&a);
        CHECK(L->pack(a) == SR_OK);
        sr_default_scene(&b);
        std::memset(b.texture_sizes, 0, sizeof b.texture_sizes);
        std::memset(b.max_texture_size, 0, sizeof b.max_texture_size);
        CHECK(std::memcmp(&a, &b, sizeof a) == 0);
        L->clear();
    }
    // material deduplication by pointer, indices from 1; null -> default material
    {
        Material m;
        m.setColor(vec4(1.f, 0.f, 0.f, 1.f));
        m.setInvertUvX(true);
        Sphere s1(vec3(1.f, 0.f, 0.f)), s2(vec3(2.f, 0.f, 0.f));
        Box bx;
        s1.setMaterial(&m);
        s2.setMaterial(&m);  // same pointer -> same index
        std::vector<const MaterialObject*> objs = {&s1, &bx, &s2};
        sr_scene s;
        CHECK(packScene(objs, {}, s) == SR_OK);
        CHECK(s.num_objects == 3);
        CHECK(s.objects[0].material_index == 1 && s.objects[1].material_index == 2 && s.objects[2].material_index == 1);
        CHECK(s.objects[0].index == 0 && s.objects[2].index == 1 && s.objects[1].index == 0);
        CHECK(s.spheres[1].transform.pos[0] == 2.f);
        CHECK(s.materials[1].color[0] == 1.f);
        CHECK(s.materials[1].invert_uv_x == 1 && s.materials[1].invert_uv_y == 1);  // material.cpp:120 quirk
        CHECK(s.materials[2].color[0] == 0.5f);  // default material for the box
    }
    // capacity: a 4th sphere overflows spheres[3] (the reference drops it silently)
    {
        Sphere s[4];
        std::vector<const MaterialObject*> objs = {&s[0], &s[1], &s[2], &s[3]};
        sr_scene sc;
        CHECK(packScene(objs, {}, sc) == SR_E_CAPACITY);
        Light l[5];
        CHECK(packScene({}, {&l[0], &l[1], &l[2], &l[3], &l[4]}, sc) == SR_E_CAPACITY);
        std::vector<Material> mats(11);
        std::vector<Sphere> many(11);
        std::vector<const MaterialObject*> o2;
        for (int i = 0; i < 11; i++) {
            many[i].setMaterial(&mats[i]);
            o2.push_back(&many[i]);
        }
        CHECK(packScene(o2, {}, sc) == SR_E_CAPACITY);
    }
    // Camera: lookAt, constructor, hyperbolic fly-by ends looking at the hole
    {
        Camera c(vec3(0.f, 2.f, 15.f), -normalize(vec3(0.f, 2.f, 15.f)), vec3(1.f, 0.f, 0.f));
        sr_camera out;
        c.load(out);
        CHECK(out.fov == 90.f);
        CHECK(std::fabs(dot(c.getUp(), c.getForward())) < 1e-6f);
        c.setPos(vec3(5.f, 0.f, 0.f));
        c.lookAt();
        CHECK(std::fabs(c.getForward().x + 1.f) < 1e-6f);
        CHECK(std::fabs(length(c.getRight()) - 1.f) < 1e-6f);
        c.hyperbolicTrajectory(30.f, 10.f, 0.5f);  // mid-way: closest approach
        float r = length(c.getPos());
        CHECK(std::fabs(r - 10.f) < 1e-3f);
        vec3 toHole = normalize(vec3(0.f, 0.f, 0.f) - c.getPos());
        CHECK(dot(toHole, c.getForward()) > 0.9999f);
        c.hyperbolicTrajectory(30.f, 10.f, 0.f);
        CHECK(std::fabs(length(c.getPos()) - 30.f) < 1e-2f);
    }
    // loadTextureArray padding: RGB layer gets alpha 255 inside, 0 outside
    {
        std::vector<unsigned char> rgb(2 * 3 * 3, 7), rgba(4 * 2 * 4, 9);
        DecodedImage a{rgb.data(), 2, 3, 3}, b{rgba.data(), 4, 2, 4};
        TextureArray ta;
        sr_scene sc;
        sr_scene_clear(&sc);
        CHECK(packTextureArray({a, b}, ta, sc) == SR_OK);
        CHECK(ta.width == 4 && ta.height == 3 && ta.layers == 2 && ta.channels == 4);
        const unsigned char* p = ta.pixels.data();
        CHECK(p[0] == 7 && p[3] == 255);                 // layer 0, (0,0) inside
        CHECK(p[(0 * 4 + 3) * 4 + 3] == 0);              // layer 0, (3,0) padding
        CHECK(p[(2 * 4 + 1) * 4 + 3] == 255);            // layer 0, (1,2) inside
        const unsigned char* q = p + 4 * 3 * 4;
        CHECK(q[3] == 9 && q[(2 * 4 + 0) * 4 + 3] == 0);  // layer 1, row 2 is padding
        CHECK(sc.texture_sizes[0][0] == 2.f && sc.texture_sizes[1][1] == 2.f);
        CHECK(sc.max_texture_size[0] == 4.f && sc.max_texture_size[1] == 3.f);
    }
    // press-R: exactly radial ray -> two points
    {
        Camera c(vec3(0.f, 0.f, 15.f));
        c.setForward(vec3(0.f, 0.f, -1.f));
        std::vector<vec3> pts = calculateTestRayPoints(c, 2000, 2);
        CHECK(pts.size() == 2 && pts[1].z == 13.f);
    }
    if (failures == 0) std::printf("ALL OK\n");
    return failures == 0 ? 0 : 1;
}
