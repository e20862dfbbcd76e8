// scene.cpp — host-side scene model (see include/sr/scene.hpp). Mirrors the
// reference's src/lib/Objects/* and ObjectLoader; packing replaces the GL
// uniform uploads. Built with -ffp-contract=off so float bits match glm's.
#include "sr/scene.hpp"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>

namespace sr {

namespace {

void putVec3(float* dst, vec3 v) {
    dst[0] = v.x;
    dst[1] = v.y;
    dst[2] = v.z;
}

// materialObject.cpp:3 — the shared default material for objects without one
const Material& defaultMaterial() {
    static const Material m;
    return m;
}

}  // namespace

// ---- Transform (transform.cpp:58-69: pos + column-major axes) -------------
void Transform::packTransform(sr_transform& out) const {
    putVec3(out.pos, m_pos);
    for (int c = 0; c < 3; c++) putVec3(out.axes + 3 * c, m_axes[c]);
}

// ---- Material ---------------------------------------------------------------
Material::Material(vec4 color, float ambient, float diffuse, float specular, float shininess)
    : m_color(color), m_ambient(ambient), m_diffuse(diffuse), m_specular(specular) {
    // material.cpp:7 writes m_shininess(m_shininess): an indeterminate value in
    // the reference. The default (32) is kept and the argument ignored, which
    // is one of the values the reference may produce.
    (void)shininess;
}

void Material::packMaterial(sr_material& out) const {
    out.color[0] = m_color.x;
    out.color[1] = m_color.y;
    out.color[2] = m_color.z;
    out.color[3] = m_color.w;
    out.ambient = m_ambient;
    out.diffuse = m_diffuse;
    out.specular = m_specular;
    out.shininess = m_shininess;
    out.texture_index = m_textureIndex;
    out.normal_map_index = m_normalMapIndex;
    out.invert_uv_x = m_invertUvX;
    out.invert_uv_y = m_invertUvX;  // material.cpp:120 uploads m_invertUvX here
    out.swap_uvs = m_swapUvs;
    out.double_sided_normals = m_doubleSidedNormals;
    out.flip_normals = m_flipNormals;
}

const Material* MaterialObject::getMaterial() const {
    return m_material ? m_material : &defaultMaterial();
}

// ---- Camera (camera.cpp) ----------------------------------------------------
Camera::Camera(vec3 pos, vec3 forward, vec3 right) : Transform(pos) {
    m_axes[0] = normalize(right);
    m_axes[2] = normalize(forward);
    m_axes[1] = normalize(cross(right, forward));
}

// camera.cpp:20-33. The reference mixes double literals and ::pow/::sqrt/::cos
// (double) into float code; the narrowing points are kept.
void Camera::hyperbolicTrajectory(float initialDistance, float closestDistance, float time) {
    const vec3 baseX(0.f, 0.f, -1.f);
    const vec3 baseY((float)std::cos(M_PI / 10.), (float)std::sin(M_PI / 10.), 0.f);
    float cd2 = (float)std::pow((double)closestDistance, 2.);
    float a = -cd2 / (-initialDistance + 2 * closestDistance);
    float c = closestDistance + a;
    float b = (float)std::sqrt((double)cd2 + 2. * (double)a * (double)closestDistance);
    float eased = (float)((1. - std::cos((double)time * M_PI)) / 2.);
    float x = (float)(-(double)initialDistance + 2. * (double)eased * (double)initialDistance);
    float y = (float)((double)c -
                      (double)a * std::sqrt(1. + std::pow((double)(x / b), 2.)));
    m_pos = x * baseX + y * baseY;
    lookAt();
}

// camera.cpp:35-39
void Camera::lookAt(vec3 point) {
    m_axes[2] = normalize(point - m_pos);
    m_axes[0] = normalize(cross(m_axes[2], vec3(0.f, 1.f, 0.f)));
    m_axes[1] = normalize(cross(m_axes[0], m_axes[2]));
}

void Camera::load(sr_camera& out) const {
    packTransform(out.transform);
    out.fov = m_fov;
}

// ---- Light (light.cpp:28-45) -----------------------------------------------
void Light::packLight(sr_light& out) const {
    packTransform(out.transform);
    putVec3(out.color, m_color);
    out.intensity = m_intensity;
    out.attenuation_constant = m_attenuationConstant;
    out.attenuation_linear = m_attenuationLinear;
    out.attenuation_quadratic = m_attenuationQuadratic;
}

// ---- shapes: per-type array slots (sphere.cpp:15-24 ... box.cpp:28-41) -----
int Sphere::packObject(sr_scene& s, int k) const {
    if (k < 0 || k >= SR_MAX_SPHERES) return SR_E_CAPACITY;
    packTransform(s.spheres[k].transform);
    s.spheres[k].radius = m_radius;
    return SR_OK;
}

void Plane::packPlane(sr_plane& out) const {
    packTransform(out.transform);
    out.texture_offset[0] = m_textureOffset.x;
    out.texture_offset[1] = m_textureOffset.y;
    out.repeat_texture = m_repeatTexture;
    out.texture_size[0] = m_textureSize.x;
    out.texture_size[1] = m_textureSize.y;
}

int Plane::packObject(sr_scene& s, int k) const {
    if (k < 0 || k >= SR_MAX_PLANES) return SR_E_CAPACITY;
    packPlane(s.planes[k]);
    return SR_OK;
}

int Disk::packObject(sr_scene& s, int k) const {
    if (k < 0 || k >= SR_MAX_DISKS) return SR_E_CAPACITY;
    packPlane(s.disks[k].plane);
    s.disks[k].radius = m_radius;
    return SR_OK;
}

int HollowDisk::packObject(sr_scene& s, int k) const {
    if (k < 0 || k >= SR_MAX_HOLLOW_DISKS) return SR_E_CAPACITY;
    packPlane(s.hollow_disks[k].plane);
    s.hollow_disks[k].inner_radius = m_innerRadius;
    s.hollow_disks[k].outer_radius = m_outerRadius;
    return SR_OK;
}

int LateralCylinder::packObject(sr_scene& s, int k) const {
    if (k < 0 || k >= SR_MAX_CYLINDERS) return SR_E_CAPACITY;
    packTransform(s.cylinders[k].transform);
    s.cylinders[k].height = m_height;
    s.cylinders[k].radius = m_radius;
    return SR_OK;
}

int Rectangle::packObject(sr_scene& s, int k) const {
    if (k < 0 || k >= SR_MAX_RECTANGLES) return SR_E_CAPACITY;
    packPlane(s.rectangles[k].plane);
    s.rectangles[k].width = m_width;
    s.rectangles[k].height = m_height;
    return SR_OK;
}

int Box::packObject(sr_scene& s, int k) const {
    if (k < 0 || k >= SR_MAX_BOXES) return SR_E_CAPACITY;
    packTransform(s.boxes[k].transform);
    s.boxes[k].width = m_width;
    s.boxes[k].depth = m_depth;
    s.boxes[k].height = m_height;
    return SR_OK;
}

// ---- ObjectLoader (objectLoader.cpp) ---------------------------------------
ObjectLoader* ObjectLoader::m_instance = nullptr;
std::mutex ObjectLoader::m_mutex;

ObjectLoader* ObjectLoader::getInstance() {
    std::lock_guard<std::mutex> lock(m_mutex);
    if (!m_instance) m_instance = new ObjectLoader();
    return m_instance;
}

void ObjectLoader::clear() {
    m_objects.clear();
    m_lights.clear();
}

int packScene(const std::vector<const MaterialObject*>& objects,
              const std::vector<const Light*>& lights, sr_scene& out) {
    sr_scene_clear(&out);
    if (objects.size() > (size_t)SR_MAX_OBJECTS || lights.size() > (size_t)SR_MAX_LIGHTS)
        return SR_E_CAPACITY;
    // objectLoader.cpp:34-42: per-type running indices, materials keyed by
    // pointer. `matMap[p]` default-inserts 0 before size() is read, so the
    // first material gets index 1 (materials[0] is never written).
    std::map<const Material*, int> matMap;
    int typeIndex[7] = {0, 0, 0, 0, 0, 0, 0};
    out.num_objects = (int32_t)objects.size();
    for (size_t i = 0; i < objects.size(); i++) {
        const MaterialObject* o = objects[i];
        int type = (int)o->getType();
        if (type < SPHERE || type > BOX) return SR_E_INVALID;
        const Material* p = o->getMaterial();
        int matIndex;
        if (!matMap[p]) {
            matIndex = (int)matMap.size();
            matMap[p] = matIndex;
            if (matIndex >= SR_MAX_MATERIALS) return SR_E_CAPACITY;
            p->packMaterial(out.materials[matIndex]);
        } else {
            matIndex = matMap[p];
        }
        int rc = o->packObject(out, typeIndex[type]);
        if (rc != SR_OK) return rc;
        out.objects[i].type = type;
        out.objects[i].index = typeIndex[type];
        out.objects[i].material_index = matIndex;
        typeIndex[type]++;
    }
    out.num_lights = (int32_t)lights.size();
    for (size_t i = 0; i < lights.size(); i++) lights[i]->packLight(out.lights[i]);
    return SR_OK;
}

int ObjectLoader::pack(sr_scene& out) const {
    std::vector<const MaterialObject*> objs(m_objects.begin(), m_objects.end());
    std::vector<const Light*> lights(m_lights.begin(), m_lights.end());
    // texture sizes belong to the texture upload; keep what the caller set
    float ts[SR_MAX_TEXTURES][2], mts[2];
    std::memcpy(ts, out.texture_sizes, sizeof ts);
    std::memcpy(mts, out.max_texture_size, sizeof mts);
    int rc = packScene(objs, lights, out);
    std::memcpy(out.texture_sizes, ts, sizeof ts);
    std::memcpy(out.max_texture_size, mts, sizeof mts);
    return rc;
}

int ObjectLoader::load(sr_ctx* ctx) const {
    sr_scene s;
    sr_scene_clear(&s);
    int rc = pack(s);
    if (rc != SR_OK) return rc;
    return sr_set_scene(ctx, &s);
}

// ---- texture array padding (image_utils.cpp:42-117) ------------------------
int packTextureArray(const std::vector<DecodedImage>& images, TextureArray& out, sr_scene& scene) {
    int maxW = 0, maxH = 0, maxC = 0;
    for (const DecodedImage& im : images) {
        if (!im.data) continue;  // a failed decode is skipped (image_utils.cpp:59-61)
        maxW = std::max(maxW, im.width);
        maxH = std::max(maxH, im.height);
        maxC = std::max(maxC, im.channels);
    }
    scene.max_texture_size[0] = (float)maxW;
    scene.max_texture_size[1] = (float)maxH;
    if (maxW == 0 || maxH == 0 || maxC == 0) return SR_E_INVALID;
    if (images.size() > (size_t)SR_MAX_TEXTURES) return SR_E_CAPACITY;
    // GL_RGBA when the widest source has 4 channels, else GL_RGB
    int outC = maxC == 4 ? 4 : 3;
    out.width = maxW;
    out.height = maxH;
    out.layers = (int)images.size();
    out.channels = outC;
    size_t layerBytes = (size_t)maxW * maxH * outC;
    out.pixels.assign(layerBytes * images.size(), 0);
    for (size_t i = 0; i < images.size(); i++) {
        const DecodedImage& im = images[i];
        if (!im.data) continue;
        unsigned char* dst = out.pixels.data() + layerBytes * i;
        for (int y = 0; y < im.height; y++) {
            for (int x = 0; x < im.width; x++) {
                const unsigned char* s = im.data + ((size_t)y * im.width + x) * im.channels;
                unsigned char* d = dst + ((size_t)y * maxW + x) * outC;
                for (int c = 0; c < outC; c++) d[c] = c < im.channels ? s[c] : (c == 3 ? 255 : 0);
            }
        }
        scene.texture_sizes[i][0] = (float)im.width;
        scene.texture_sizes[i][1] = (float)im.height;
    }
    return SR_OK;
}

// ---- press-R test ray (src/main.cpp:73-124) ---------------------------------
namespace {

// The reference writes these with double literals in float code; every
// intermediate below is evaluated in double and narrowed where C++ narrows it.
float binetAccel(float u) { return (float)((double)(-u) * (1.0 - 1.5 * (double)u)); }

struct Increment {
    float du, dv;
};

Increment rk4Increment(float u, float v, float h) {
    const double hd = h;
    float k1 = v;
    float l1 = binetAccel(u);
    float k2 = (float)((double)v + 0.5 * (double)l1 * hd);
    float l2 = binetAccel((float)((double)u + 0.5 * (double)k1 * hd));
    float k3 = (float)((double)v + 0.5 * (double)l2 * hd);
    float l3 = binetAccel((float)((double)u + 0.5 * (double)k2 * hd));
    float k4 = v + l3 * h;
    float l4 = binetAccel(u + k3 * h);
    Increment r;
    r.du = (float)(hd / 6. * ((double)k1 + 2. * (double)k2 + 2. * (double)k3 + (double)k4));
    r.dv = (float)(hd / 6. * ((double)l1 + 2. * (double)l2 + 2. * (double)l3 + (double)l4));
    return r;
}

}  // namespace

std::vector<vec3> calculateTestRayPoints(const Camera& cam, int maxSteps, int maxRevolutions) {
    vec3 dir = cam.getForward();
    vec3 origin = cam.getPos() + dir * 1.0f;  // TEST_RAY_OFFSET
    vec3 n = normalize(origin);
    vec3 t = normalize(cross(cross(n, dir), n));
    float u = (float)(1. / (double)length(origin));
    float du = -u * dot(dir, n) / dot(dir, t);
    // src/main.cpp:104: unqualified abs(float) binds ::abs(int) there
    if (std::abs((int)dot(dir, n)) >= 1. - 0.000001) return {origin, origin + dir};
    std::vector<vec3> out{origin};
    const double maxAngle = 2. * (double)(float)maxRevolutions * M_PI;
    float phi = 0.f;
    for (int i = 0; i < maxSteps; i++) {
        float h = (float)((maxAngle - (double)phi) / (double)(float)(maxSteps - i));
        phi += h;
        Increment inc = rk4Increment(u, du, h);
        u += inc.du;
        if (u < 0.f || u > 1.f) break;  // checked before du is advanced
        du += inc.dv;
        out.push_back(((float)std::cos((double)phi) * n + (float)std::sin((double)phi) * t) / u);
    }
    return out;
}

// ---- the app's default scene (src/main.cpp:222-268) --------------------------
DefaultScene::DefaultScene()
    : cam(vec3(0.f, 2.f, 15.f), -normalize(vec3(0.f, 2.f, 15.f)), vec3(1.f, 0.f, 0.f)),
      sphere(vec3(-10.f, 0.f, 0.f)) {
    mat1.setTextureIndex(0);
    sphere.setMaterial(&mat1);
    disk.setRadius(2.f);
    disk.setPos(vec3(0.f, 0.f, -10.f));
    disk.setAxes(angleAxis((float)M_PI / 4.f, normalize(vec3(1.f, 1.f, 1.f))));
    disk.setMaterial(&mat1);
    accretionDisk.setMaterial(&mat1);
    cyl.setPos(vec3(0.f, 10.f, 0.f));
    cyl.setHeight(5.f);
    cyl.setRadius(2.f);
    cyl.setMaterial(&mat1);
    rect.setPos(vec3(0.f, 0.f, 10.f));
    rect.setWidth(3.f);
    rect.setHeight(2.f);
    rect.setMaterial(&mat1);
    mat2.setTextureIndex(1);
    box.setPos(vec3(10.f, 0.f, 0.f));
    box.setMaterial(&mat2);
    light.setIntensity(8.f);
}

std::vector<const MaterialObject*> DefaultScene::objects() const {
    return {&sphere, &disk, &accretionDisk, &cyl, &rect, &box};
}

std::vector<const Light*> DefaultScene::lights() const { return {&light}; }

void DefaultScene::registerWith(ObjectLoader& loader) {
    loader.addObject(&sphere);
    loader.addObject(&disk);
    loader.addObject(&accretionDisk);
    loader.addObject(&cyl);
    loader.addObject(&rect);
    loader.addObject(&box);
    loader.addLight(&light);
}

}  // namespace sr

// ---- C-ABI pieces that live on the host side --------------------------------
extern "C" {

void sr_scene_clear(sr_scene* out) {
    if (out) std::memset(out, 0, sizeof(*out));
}

void sr_params_default(sr_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->max_steps = 100;      // frag:19
    p->max_revolutions = 2;  // frag:20 (the app's float upload is rejected)
    p->u_f = 0.01f;          // frag:22
    p->crosshair = 0;
    p->raytrace_type = SR_RAYTRACE_CURVED;
    p->curved_percentage = 0.5f;  // frag:37
    p->percent_black = 0.75f;     // frag:39
    p->time = 0.f;
    p->filter_mode = SR_FILTER_LERP;
}

void sr_test_ray_default(sr_test_ray* t) {
    if (!t) return;
    std::memset(t, 0, sizeof(*t));
    t->visible = 0;               // frag:187
    t->radius = 0.025f;           // frag:189
    t->extended_length = 1000.f;  // frag:190
    t->curved_color[0] = 1.f;     // frag:191
    t->curved_color[3] = 1.f;
    t->flat_color[1] = 1.f;  // frag:192
    t->flat_color[3] = 1.f;
}

void sr_default_scene(sr_scene* out) {
    if (!out) return;
    sr::DefaultScene d;
    sr::packScene(d.objects(), d.lights(), *out);
    // loadTextureArray({uv_checker.jpg 600x600 RGB, cubemap.png 1601x1201 RGBA})
    out->texture_sizes[0][0] = 600.f;
    out->texture_sizes[0][1] = 600.f;
    out->texture_sizes[1][0] = 1601.f;
    out->texture_sizes[1][1] = 1201.f;
    out->max_texture_size[0] = 1601.f;
    out->max_texture_size[1] = 1201.f;
}

void sr_default_camera(sr_camera* out) {
    if (!out) return;
    sr::DefaultScene d;
    d.cam.load(*out);
}

int sr_camera_hyperbolic_trajectory(sr_camera* cam, float initial_distance, float closest_distance, float time) {
    if (!cam) return SR_E_INVALID;
    const float* a = cam->transform.axes;
    sr::Camera c(sr::vec3(cam->transform.pos[0], cam->transform.pos[1], cam->transform.pos[2]),
                 sr::vec3(a[6], a[7], a[8]), sr::vec3(a[0], a[1], a[2]));
    c.setFov(cam->fov);
    c.hyperbolicTrajectory(initial_distance, closest_distance, time);
    c.load(*cam);
    return SR_OK;
}

int sr_test_ray_points(const float cam_pos[3], const float cam_forward[3], int max_steps,
                       int max_revolutions, float* out_xyz, int max_points, int* out_count) {
    if (!cam_pos || !cam_forward || max_steps < 0 || (max_points > 0 && !out_xyz))
        return SR_E_INVALID;
    sr::Camera cam(sr::vec3(cam_pos[0], cam_pos[1], cam_pos[2]));
    cam.setForward(sr::vec3(cam_forward[0], cam_forward[1], cam_forward[2]));
    std::vector<sr::vec3> pts = sr::calculateTestRayPoints(cam, max_steps, max_revolutions);
    int n = (int)pts.size();
    for (int i = 0; i < n && i < max_points; i++) {
        out_xyz[3 * i + 0] = pts[i].x;
        out_xyz[3 * i + 1] = pts[i].y;
        out_xyz[3 * i + 2] = pts[i].z;
    }
    if (out_count) *out_count = n;
    return SR_OK;
}

}  // extern "C"
