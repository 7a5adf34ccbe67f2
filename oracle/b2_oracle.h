/*
 * oracle/b2_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * Plain-C restatement of the subset of Box2D 2.3 (box2d-py==2.3.8,
 * /root/reference/requirements.txt:4) that the reference's hot path exercises:
 * one dynamic box (the car) against ~730 static boxes (the walls) in a private
 * b2World per car (src/car_physics.py:83).  Box2D itself is a third-party
 * dependency that is NOT vendored under /root/reference and is not installed
 * here, so this file restates the published Box2D 2.3.x algorithms:
 *   b2World::Step / Solve / SolveTOI, b2Island::Solve / SolveTOI,
 *   b2ContactSolver (sequential impulses + 2-point block solver),
 *   b2CollidePolygons, b2TimeOfImpact / b2Distance (GJK),
 *   b2DynamicTree fat-AABB proxy semantics, b2PolygonShape::RayCast.
 * PARITY AT THIS BOUNDARY IS UNPINNED (no Box2D binary or source exists in
 * this container); see DESIGN.md "Oracle" for what IS pinned.
 *
 * float32 arithmetic exactly as the C++ source (no FMA contraction: build with
 * -ffp-contract=off).  b2Rot::Set uses glibc sinf/cosf, like the reference.
 */
#ifndef NASCAR_B2_ORACLE_H
#define NASCAR_B2_ORACLE_H
#include <stdint.h>

#define OB_MAXC 24          /* contacts kept per car world (overflow is flagged) */

typedef struct { float x, y; } ov2;
typedef struct { float s, c; } orot;
typedef struct { ov2 p; orot q; } oxf;
typedef struct { ov2 lo, hi; } oaabb;

typedef struct {
    ov2 localPoint; float normalImpulse, tangentImpulse; uint32_t id;
} ompt;

typedef struct {
    int type;            /* 1 = e_faceA, 2 = e_faceB */
    ov2 localNormal, localPoint;
    int pointCount;
    ompt pts[2];
} omanifold;

enum { OC_TOUCH = 1, OC_ENABLED = 2, OC_ISLAND = 4, OC_TOI = 8 };

typedef struct {
    int wall; int flags; omanifold m; float toi; int toiCount;
} ocontact;

/* static wall table of one track (built by the wall builder, see nascar_oracle.c) */
typedef struct {
    int n;
    ov2 *p; float *angle; orot *q; float *hx, *hy; oaabb *fat; int *key;
} owalls;

/* one private b2World: the car body + its contact list + listener hooks */
typedef struct {
    /* body */
    ov2 c; float a; ov2 v; float w; oxf xf; float sleepTime; int awake;
    ov2 force; float torque;
    ov2 c0; float a0; float alpha0;
    oaabb fat;                 /* car proxy fat AABB (tree node aabb) */
    int moved;                 /* proxy in move buffer */
    /* contact list, index 0 == head of b2World::m_contactList */
    ocontact ct[OB_MAXC]; int nct; int overflow;
    float inv_dt0;
} oworld;

/* contact-listener callbacks (src/car_physics.py:693-864), implemented by the env */
typedef struct {
    void *user;
    void (*begin)(void *user, int wall, ov2 normal);
    void (*end)(void *user, int wall);
    void (*post)(void *user, int count, const float *normalImpulses);
} olistener;

void ob_world_init(oworld *w, const owalls *W, ov2 pos, float angle);
void ob_apply_force(oworld *w, ov2 f, ov2 point);
void ob_apply_force_center(oworld *w, ov2 f);
void ob_apply_torque(oworld *w, float t);
void ob_step(oworld *w, const owalls *W, const olistener *L, float dt, int velIters, int posIters);
void ob_set_transform(oworld *w, const owalls *W, ov2 pos, float angle);
float ob_raycast(const owalls *W, ov2 p1, ov2 p2);   /* returns min hit fraction or -1 */
int ob_query_on_wall(const owalls *W, double px, double py, double radius);
void ob_rot_set(orot *q, float a);
float ob_sinf(float x);
float ob_cosf(float x);

#endif
