// scene.hpp — host-side mirror of the reference's scene model
// (src/lib/Objects/*, src/lib/ObjectLoader/*, Camera::hyperbolicTrajectory,
// calculateTestRayPoints). Same class names, setters, defaults and quirks; the
// GL `loadShader(GLuint program, std::string prefix)` upload is replaced by
// packing into the C-ABI structs of sr.h, and ObjectLoader::load(program) by
// ObjectLoader::load(sr_ctx*) (a snapshot copy into the device context).
#ifndef SR_SCENE_HPP
#define SR_SCENE_HPP

#include <mutex>
#include <string>
#include <vector>

#include "sr.h"
#include "vecmath.hpp"

namespace sr {

// object.h:7-19
enum ObjectType {
    UNKNOWN = -999,
    MATERIAL = -3,
    CAMERA = -2,
    LIGHT = -1,
    SPHERE,
    PLANE,
    DISK,
    HOLLOW_DISK,
    LATERAL_CYLINDER,
    RECTANGLE,
    BOX
};

// camera.h:14-19
enum RaytraceType { CURVED, FLAT, HALF_WIDTH, HALF_HEIGHT };

// camera.h:7-12
constexpr float DEFAULT_FOV = 90.f;
constexpr float HYPERBOLIC_TRAJECTORY_DURATION = 5.f;

// src/main.cpp:66-71 (app compile-time knobs)
constexpr float PERCENT_BLACK = 0.75f;
constexpr int MAX_STEPS = 100;
constexpr int MAX_REVOLUTIONS = 2;

class Object {
public:
    virtual ~Object() = default;
    virtual ObjectType getType() const { return UNKNOWN; }
};

// transform.h/.cpp
class Transform : public virtual Object {
public:
    Transform() = default;
    explicit Transform(vec3 pos) : m_pos(pos) {}

    vec3 getPos() const { return m_pos; }
    void setPos(vec3 p) { m_pos = p; }
    mat3 getAxes() const { return m_axes; }
    void setAxes(const mat3& a) { m_axes = a; }
    void setAxes(const quat& rot) { m_axes = toMat3(rot); }
    vec3 getForward() const { return m_axes[2]; }
    void setForward(vec3 v) { m_axes[2] = v; }
    vec3 getRight() const { return m_axes[0]; }
    void setRight(vec3 v) { m_axes[0] = v; }
    vec3 getUp() const { return m_axes[1]; }
    void setUp(vec3 v) { m_axes[1] = v; }
    void calculateForward() { m_axes[2] = normalize(cross(m_axes[0], m_axes[1])); }
    void calculateRight() { m_axes[0] = normalize(cross(m_axes[1], m_axes[2])); }
    void calculateUp() { m_axes[1] = normalize(cross(m_axes[2], m_axes[0])); }

    // replaces Transform::loadShader (transform.cpp:58-69)
    void packTransform(sr_transform& out) const;

protected:
    vec3 m_pos{0.f, 0.f, 0.f};
    mat3 m_axes{};
};

// material.h/.cpp — defaults material.h:53-64
class Material : public virtual Object {
public:
    Material() = default;
    explicit Material(vec4 color) : m_color(color) {}
    // material.cpp:6-7: the reference initialises m_shininess from itself; the
    // value is indeterminate there. We keep the default (32) and flag it.
    Material(vec4 color, float ambient, float diffuse, float specular, float shininess);

    vec4 getColor() const { return m_color; }
    void setColor(vec4 c) { m_color = c; }
    float getAmbient() const { return m_ambient; }
    void setAmbient(float v) { m_ambient = v; }
    float getDiffuse() const { return m_diffuse; }
    void setDiffuse(float v) { m_diffuse = v; }
    float getSpecular() const { return m_specular; }
    void setSpecular(float v) { m_specular = v; }
    float getShininess() const { return m_shininess; }
    void setShininess(float v) { m_shininess = v; }
    int getTextureIndex() const { return m_textureIndex; }
    void setTextureIndex(int i) { m_textureIndex = i; }
    int getNormalMapIndex() const { return m_normalMapIndex; }
    void setNormalMapIndex(int i) { m_normalMapIndex = i; }
    bool getInvertUvX() const { return m_invertUvX; }
    void setInvertUvX(bool b) { m_invertUvX = b; }
    bool getInvertUvY() const { return m_invertUvY; }
    void setInvertUvY(bool b) { m_invertUvY = b; }
    bool getSwapUvs() const { return m_swapUvs; }
    void setSwapUvs(bool b) { m_swapUvs = b; }
    bool getDoubleSidedNormals() const { return m_doubleSidedNormals; }
    void setDoubleSidedNormals(bool b) { m_doubleSidedNormals = b; }
    bool getFlipNormals() const { return m_flipNormals; }
    void setFlipNormals(bool b) { m_flipNormals = b; }

    // replaces Material::loadShader (material.cpp:93-124) including its quirk:
    // invert_uv_y receives m_invertUvX (material.cpp:120).
    void packMaterial(sr_material& out) const;
    ObjectType getType() const override { return MATERIAL; }

private:
    vec4 m_color{0.5f, 0.f, 0.5f, 1.f};
    float m_ambient = 0.1f;
    float m_diffuse = 0.9f;
    float m_specular = 0.5f;
    float m_shininess = 32.f;
    int m_textureIndex = -1;
    int m_normalMapIndex = -1;
    bool m_invertUvX = false;
    bool m_invertUvY = false;
    bool m_swapUvs = false;
    bool m_doubleSidedNormals = true;
    bool m_flipNormals = false;
};

// materialObject.h/.cpp: a null material means the static default material.
class MaterialObject : public virtual Object {
public:
    MaterialObject() = default;
    explicit MaterialObject(Material* mat) : m_material(mat) {}
    const Material* getMaterial() const;
    void setMaterial(Material* mat) { m_material = mat; }
    // writes this object into its per-type array slot of the scene
    virtual int packObject(sr_scene& scene, int index) const = 0;

protected:
    Material* m_material = nullptr;
};

// camera.h/.cpp
class Camera : public Transform {
public:
    Camera() = default;
    explicit Camera(vec3 pos) : Transform(pos) {}
    Camera(vec3 pos, vec3 forward, vec3 right);

    void setFov(float fov) { m_fov = fov; }
    float getFov() const { return m_fov; }
    void hyperbolicTrajectory(float initialDistance, float closestDistance, float time);
    void lookAt(vec3 point = vec3(0.f, 0.f, 0.f));
    // replaces Camera::loadShader(program) (camera.cpp:41-50)
    void load(sr_camera& out) const;
    ObjectType getType() const override { return CAMERA; }

private:
    float m_fov = DEFAULT_FOV;
};

// light.h/.cpp — default light.cpp:4
class Light : public Transform {
public:
    Light() : Light(vec3(10.f, 10.f, 10.f), vec3(1.f, 1.f, 1.f), 2.5f) {}
    Light(vec3 pos, vec3 color, float intensity, float attenuationConstant = 1.f,
          float attenuationLinear = 0.09f, float attenuationQuadratic = 0.032f)
        : Transform(pos),
          m_color(color),
          m_intensity(intensity),
          m_attenuationConstant(attenuationConstant),
          m_attenuationLinear(attenuationLinear),
          m_attenuationQuadratic(attenuationQuadratic) {}

    vec3 getColor() const { return m_color; }
    void setColor(vec3 c) { m_color = c; }
    float getIntensity() const { return m_intensity; }
    void setIntensity(float v) { m_intensity = v; }
    float getAttenuationConstant() const { return m_attenuationConstant; }
    void setAttenuationConstant(float v) { m_attenuationConstant = v; }
    float getAttenuationLinear() const { return m_attenuationLinear; }
    void setAttenuationLinear(float v) { m_attenuationLinear = v; }
    float getAttenuationQuadratic() const { return m_attenuationQuadratic; }
    void setAttenuationQuadratic(float v) { m_attenuationQuadratic = v; }
    void packLight(sr_light& out) const;
    ObjectType getType() const override { return LIGHT; }

private:
    vec3 m_color;
    float m_intensity;
    float m_attenuationConstant;
    float m_attenuationLinear;
    float m_attenuationQuadratic;
};

// sphere.h/.cpp
class Sphere : public MaterialObject, public Transform {
public:
    Sphere() = default;
    explicit Sphere(vec3 pos) : Transform(pos) {}
    Sphere(vec3 pos, float radius) : Transform(pos), m_radius(radius) {}
    float getRadius() const { return m_radius; }
    void setRadius(float r) { m_radius = r; }
    int packObject(sr_scene& scene, int index) const override;
    ObjectType getType() const override { return SPHERE; }

private:
    float m_radius = 1.f;
};

// plane.h/.cpp
class Plane : public MaterialObject, public Transform {
public:
    Plane() = default;
    explicit Plane(vec3 pos) : Transform(pos) {}
    vec2 getTextureSize() const { return m_textureSize; }
    void setTextureSize(vec2 s) { m_textureSize = s; }
    vec2 getTextureOffset() const { return m_textureOffset; }
    void setTextureOffset(vec2 o) { m_textureOffset = o; }
    bool getRepeatTexture() const { return m_repeatTexture; }
    void setRepeatTexture(bool b) { m_repeatTexture = b; }
    int packObject(sr_scene& scene, int index) const override;
    ObjectType getType() const override { return PLANE; }

protected:
    void packPlane(sr_plane& out) const;

private:
    vec2 m_textureSize{1.f, 1.f};
    vec2 m_textureOffset{0.f, 0.f};
    bool m_repeatTexture = true;
};

// disk.h/.cpp
class Disk : public Plane {
public:
    Disk() = default;
    explicit Disk(vec3 pos) : Plane(pos) {}
    float getRadius() const { return m_radius; }
    void setRadius(float r) { m_radius = r; }
    int packObject(sr_scene& scene, int index) const override;
    ObjectType getType() const override { return DISK; }

private:
    float m_radius = 1.f;
};

// hollowDisk.h/.cpp
class HollowDisk : public Plane {
public:
    HollowDisk() = default;
    explicit HollowDisk(vec3 pos) : Plane(pos) {}
    float getInnerRadius() const { return m_innerRadius; }
    void setInnerRadius(float r) { m_innerRadius = r; }
    float getOuterRadius() const { return m_outerRadius; }
    void setOuterRadius(float r) { m_outerRadius = r; }
    int packObject(sr_scene& scene, int index) const override;
    ObjectType getType() const override { return HOLLOW_DISK; }

private:
    float m_innerRadius = 2.5f;
    float m_outerRadius = 5.f;
};

// lateralCylinder.h/.cpp
class LateralCylinder : public MaterialObject, public Transform {
public:
    LateralCylinder() = default;
    float getHeight() const { return m_height; }
    void setHeight(float h) { m_height = h; }
    float getRadius() const { return m_radius; }
    void setRadius(float r) { m_radius = r; }
    int packObject(sr_scene& scene, int index) const override;
    ObjectType getType() const override { return LATERAL_CYLINDER; }

private:
    float m_height = 5.f;
    float m_radius = 1.f;
};

// rectangle.h/.cpp
class Rectangle : public Plane {
public:
    Rectangle() = default;
    explicit Rectangle(vec3 pos) : Plane(pos) {}
    float getWidth() const { return m_width; }
    void setWidth(float w) { m_width = w; }
    float getHeight() const { return m_height; }
    void setHeight(float h) { m_height = h; }
    int packObject(sr_scene& scene, int index) const override;
    ObjectType getType() const override { return RECTANGLE; }

private:
    float m_width = 1.f;
    float m_height = 1.f;
};

// box.h/.cpp
class Box : public MaterialObject, public Transform {
public:
    Box() = default;
    explicit Box(vec3 pos) : Transform(pos) {}
    float getWidth() const { return m_width; }
    void setWidth(float w) { m_width = w; }
    float getDepth() const { return m_depth; }
    void setDepth(float d) { m_depth = d; }
    float getHeight() const { return m_height; }
    void setHeight(float h) { m_height = h; }
    int packObject(sr_scene& scene, int index) const override;
    ObjectType getType() const override { return BOX; }

private:
    float m_width = 1.f;
    float m_depth = 1.f;
    float m_height = 1.f;
};

// objectLoader.h/.cpp — singleton holding non-owning pointers.
class ObjectLoader {
public:
    ObjectLoader(ObjectLoader&) = delete;
    void operator=(const ObjectLoader&) = delete;
    static ObjectLoader* getInstance();

    void addLight(Light* light) { m_lights.push_back(light); }
    void addObject(MaterialObject* object) { m_objects.push_back(object); }
    void clear();

    // Flattens the registered objects exactly as ObjectLoader::load
    // (objectLoader.cpp:27-109) writes GLSL uniforms: per-type running
    // indices, materials deduplicated by pointer with indices starting at 1,
    // objects[i] = {type, index, material_index}. Returns SR_E_CAPACITY where
    // the reference would silently drop a uniform write.
    int pack(sr_scene& out) const;
    // pack + sr_set_scene: the snapshot upload that replaces load(GLuint program)
    int load(sr_ctx* ctx) const;

protected:
    ObjectLoader() = default;
    ~ObjectLoader() = default;

private:
    static ObjectLoader* m_instance;
    static std::mutex m_mutex;
    std::vector<Light*> m_lights;
    std::vector<MaterialObject*> m_objects;
};

// The flattening rules of ObjectLoader::load as a free function (used by the
// singleton and by sr_default_scene).
int packScene(const std::vector<const MaterialObject*>& objects,
              const std::vector<const Light*>& lights, sr_scene& out);

// image_utils.cpp:42-117 — pads decoded images to the largest width/height/
// channel count (RGB sources get alpha 255 inside the image, 0 in padding) and
// records texture_sizes / max_texture_size as the reference's uniforms.
struct DecodedImage {
    const unsigned char* data = nullptr;  // rows bottom-up (stbi flip applied)
    int width = 0, height = 0, channels = 0;
};
struct TextureArray {
    std::vector<unsigned char> pixels;  // layer-major, max_w x max_h x channels
    int width = 0, height = 0, layers = 0, channels = 0;
};
int packTextureArray(const std::vector<DecodedImage>& images, TextureArray& out, sr_scene& scene);

// src/main.cpp:94-124 — the press-R test ray (CPU), MAX_STEPS/MAX_REVOLUTIONS
// as arguments.
std::vector<vec3> calculateTestRayPoints(const Camera& cam, int maxSteps = MAX_STEPS,
                                         int maxRevolutions = MAX_REVOLUTIONS);

// src/main.cpp:222-268: builds the reference's hard-coded scene into `loader`
// (objects are owned by the returned holder).
struct DefaultScene {
    Camera cam;
    Material mat1, mat2;
    Sphere sphere;
    Disk disk;
    HollowDisk accretionDisk;
    LateralCylinder cyl;
    Rectangle rect;
    Box box;
    Light light;
    DefaultScene();
    DefaultScene(const DefaultScene&) = delete;
    void registerWith(ObjectLoader& loader);
    std::vector<const MaterialObject*> objects() const;
    std::vector<const Light*> lights() const;
};

}  // namespace sr

#endif
