// ref_golden.cpp — driver that links the REFERENCE's own CPU geometry
// library (compiled from /root/reference/{Sphere,Hittable_list,Camera}.cpp
// by oracle/Makefile) and evaluates it on inputs read from stdin.
// TEST INFRASTRUCTURE ONLY: used by tests/golden/make_golden.py to produce
// the committed golden vectors; never shipped, never run on the GPU box.
//
// stdin  : nspheres / (cx cy cz r) x n / nrays t_min t_max / (o.xyz d.xyz) x nrays
//          / ncam W H / (u v) x ncam            (doubles in %.17g)
// stdout : per ray  "hit t p.xyz normal.xyz front_face index"
//          per cam  "o.xyz d.xyz"  (Camera(W,H).get_ray(u,v), Camera.h:23-26)
#include <cstdio>
#include <memory>
#include <vector>

#include "Camera.h"
#include "Hittable_list.h"
#include "Sphere.h"

namespace {
int g_last_id = -1;
// Sphere that reports which list entry produced the last accepted hit; the
// reference's hit_record has no index, Hittable_list keeps the last one.
struct IdSphere : public Sphere {
    IdSphere(Point3 c, double r, int id_) : Sphere(c, r), id(id_) {}
    bool hit(const Ray &r, double t_min, double t_max, hit_record &rec) const override {
        const bool h = Sphere::hit(r, t_min, t_max, rec);
        if (h) g_last_id = id;
        return h;
    }
    int id;
};
}  // namespace

int main() {
    int ns = 0;
    if (std::scanf("%d", &ns) != 1) return 1;
    Hittable_list world;
    for (int i = 0; i < ns; ++i) {
        double x, y, z, r;
        if (std::scanf("%lf %lf %lf %lf", &x, &y, &z, &r) != 4) return 1;
        world.add(std::make_shared<IdSphere>(Point3(x, y, z), r, i));
    }
    int nr = 0;
    double tmin, tmax;
    if (std::scanf("%d %lf %lf", &nr, &tmin, &tmax) != 3) return 1;
    for (int i = 0; i < nr; ++i) {
        double o[3], d[3];
        if (std::scanf("%lf %lf %lf %lf %lf %lf", &o[0], &o[1], &o[2], &d[0], &d[1], &d[2]) != 6) return 1;
        const Ray ray(Point3(o[0], o[1], o[2]), Vec3(d[0], d[1], d[2]));
        hit_record rec;
        g_last_id = -1;
        int winner = -1;
        // Hittable_list::hit overwrites rec only on hits; the last hit wins.
        const bool h = world.hit(ray, tmin, tmax, rec);
        if (h) {
            winner = g_last_id;  // last IdSphere::hit that returned true
            std::printf("1 %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d %d\n", rec.t, rec.p[0], rec.p[1],
                        rec.p[2], rec.normal[0], rec.normal[1], rec.normal[2], rec.front_face ? 1 : 0,
                        winner);
        } else {
            std::printf("0 0 0 0 0 0 0 0 0 -1\n");
        }
    }
    int nc = 0;
    unsigned W = 0, H = 0;
    if (std::scanf("%d %u %u", &nc, &W, &H) != 3) return 1;
    const Camera cam(W, H);
    for (int i = 0; i < nc; ++i) {
        double u, v;
        if (std::scanf("%lf %lf", &u, &v) != 2) return 1;
        const Ray r = cam.get_ray(u, v);
        std::printf("%.17g %.17g %.17g %.17g %.17g %.17g\n", r.orig[0], r.orig[1], r.orig[2], r.dir[0],
                    r.dir[1], r.dir[2]);
    }
    return 0;
}
