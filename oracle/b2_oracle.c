/*
 * oracle/b2_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 * Box2D 2.3 subset restated in plain C; see b2_oracle.h for scope and the
 * "parity unpinned" note.  Every routine names the Box2D 2.3 function it
 * follows; the reference call site for each is given in b2_oracle.h /
 * nascar_oracle.c.  Build with -O2 -ffp-contract=off (no FMA contraction).
 */
#include "b2_oracle.h"
#include <float.h>
#include <math.h>
#include <string.h>

/* ---- b2Settings.h ---- */
#define B2_PI 3.14159265359f
#define LINEAR_SLOP 0.005f
#define POLY_RADIUS (2.0f * LINEAR_SLOP)
#define AABB_EXT 0.1f
#define AABB_MULT 2.0f
#define MAX_TRANSLATION 2.0f
#define MAX_TRANSLATION_SQ (MAX_TRANSLATION * MAX_TRANSLATION)
#define MAX_ROTATION (0.5f * B2_PI)
#define MAX_ROTATION_SQ (MAX_ROTATION * MAX_ROTATION)
#define BAUMGARTE 0.2f
#define TOI_BAUMGARTE 0.75f
#define MAX_LINEAR_CORRECTION 0.2f
#define VELOCITY_THRESHOLD 1.0f
#define TIME_TO_SLEEP 0.5f
#define LINEAR_SLEEP_TOL 0.01f
#define ANGULAR_SLEEP_TOL (2.0f / 180.0f * B2_PI)
#define MAX_SUBSTEPS 8
#define MAX_TOI_CONTACTS 32
#define MAX_POLY_VERTS 8

/* car fixture (src/car.py:217-239, src/constants/car_specs.py) */
#define CAR_HX ((float)(5.042 / 2.0))
#define CAR_HY ((float)(1.996 / 2.0))
#define CAR_INV_MASS (1.0f / 1500.0f)
/* CAR_MOMENT_OF_INERTIA = m*(L^2+W^2)*0.5/12 evaluated in double, then float (SWIG) */
static float car_I(void) { return (float)(1500.0 * (5.042 * 5.042 + 1.996 * 1.996) * 0.5 / 12.0); }
#define CAR_INV_I (1.0f / car_I())
/* b2MixFriction(0.7, 0.333) / b2MixRestitution(0.1, 0.25) */
static float mix_friction(void) { return sqrtf(0.7f * 0.333f); }
#define MIX_RESTITUTION 0.25f

/* ------------------------------------------------------------------ */
/* glibc sinf/cosf, exactly what b2Rot::Set calls in the reference.     */
float ob_sinf(float x) { return sinf(x); }
float ob_cosf(float x) { return cosf(x); }
void ob_rot_set(orot *q, float a) { q->s = sinf(a); q->c = cosf(a); }

/* ---- b2Math.h ---- */
static inline ov2 V(float x, float y) { ov2 r; r.x = x; r.y = y; return r; }
static inline ov2 vadd(ov2 a, ov2 b) { return V(a.x + b.x, a.y + b.y); }
static inline ov2 vsub(ov2 a, ov2 b) { return V(a.x - b.x, a.y - b.y); }
static inline ov2 vmul(float s, ov2 a) { return V(s * a.x, s * a.y); }
static inline ov2 vneg(ov2 a) { return V(-a.x, -a.y); }
static inline float vdot(ov2 a, ov2 b) { return a.x * b.x + a.y * b.y; }
static inline float vcross(ov2 a, ov2 b) { return a.x * b.y - a.y * b.x; }
static inline ov2 vcross_vs(ov2 a, float s) { return V(s * a.y, -s * a.x); }
static inline ov2 vcross_sv(float s, ov2 a) { return V(-s * a.y, s * a.x); }
static inline float vlen(ov2 a) { return sqrtf(a.x * a.x + a.y * a.y); }
static inline float vnormalize(ov2 *a) {
    float length = vlen(*a);
    if (length < FLT_EPSILON) return 0.0f;
    float inv = 1.0f / length;
    a->x *= inv; a->y *= inv;
    return length;
}
static inline ov2 rmul(orot q, ov2 v) { return V(q.c * v.x - q.s * v.y, q.s * v.x + q.c * v.y); }
static inline ov2 rmulT(orot q, ov2 v) { return V(q.c * v.x + q.s * v.y, -q.s * v.x + q.c * v.y); }
static inline ov2 xmul(oxf T, ov2 v) {
    float x = (T.q.c * v.x - T.q.s * v.y) + T.p.x;
    float y = (T.q.s * v.x + T.q.c * v.y) + T.p.y;
    return V(x, y);
}
static inline ov2 xmulT(oxf T, ov2 v) {
    float px = v.x - T.p.x, py = v.y - T.p.y;
    return V(T.q.c * px + T.q.s * py, -T.q.s * px + T.q.c * py);
}
static inline orot rmulT_rr(orot q, orot r) {
    orot o; o.s = q.c * r.s - q.s * r.c; o.c = q.c * r.c + q.s * r.s; return o;
}
static inline oxf xmulT_xx(oxf A, oxf B) {
    oxf C; C.q = rmulT_rr(A.q, B.q); C.p = rmulT(A.q, vsub(B.p, A.p)); return C;
}
static inline float fmin_b2(float a, float b) { return a < b ? a : b; }
static inline float fmax_b2(float a, float b) { return a > b ? a : b; }
static inline float fclamp(float a, float lo, float hi) { return fmax_b2(lo, fmin_b2(a, hi)); }
static inline ov2 vmin(ov2 a, ov2 b) { return V(fmin_b2(a.x, b.x), fmin_b2(a.y, b.y)); }
static inline ov2 vmax(ov2 a, ov2 b) { return V(fmax_b2(a.x, b.x), fmax_b2(a.y, b.y)); }

/* ---- polygons: b2PolygonShape::SetAsBox(hx, hy) ---- */
typedef struct { ov2 v[4]; ov2 n[4]; int count; float radius; } opoly;
static void box(opoly *p, float hx, float hy) {
    p->count = 4; p->radius = POLY_RADIUS;
    p->v[0] = V(-hx, -hy); p->v[1] = V(hx, -hy); p->v[2] = V(hx, hy); p->v[3] = V(-hx, hy);
    p->n[0] = V(0.0f, -1.0f); p->n[1] = V(1.0f, 0.0f); p->n[2] = V(0.0f, 1.0f); p->n[3] = V(-1.0f, 0.0f);
}
static void car_poly(opoly *p) { box(p, CAR_HX, CAR_HY); }
static void wall_poly(opoly *p, const owalls *W, int j) { box(p, W->hx[j], W->hy[j]); }
static oxf wall_xf(const owalls *W, int j) { oxf t; t.p = W->p[j]; t.q = W->q[j]; return t; }

/* b2PolygonShape::ComputeAABB */
static oaabb poly_aabb(const opoly *p, oxf xf) {
    ov2 lower = xmul(xf, p->v[0]), upper = lower;
    for (int i = 1; i < p->count; ++i) { ov2 v = xmul(xf, p->v[i]); lower = vmin(lower, v); upper = vmax(upper, v); }
    ov2 r = V(p->radius, p->radius);
    oaabb a; a.lo = vsub(lower, r); a.hi = vadd(upper, r); return a;
}
/* b2TestOverlap */
static int overlap(oaabb a, oaabb b) {
    ov2 d1 = vsub(b.lo, a.hi), d2 = vsub(a.lo, b.hi);
    if (d1.x > 0.0f || d1.y > 0.0f) return 0;
    if (d2.x > 0.0f || d2.y > 0.0f) return 0;
    return 1;
}
static int contains(oaabb a, oaabb b) {
    int r = 1;
    r = r && a.lo.x <= b.lo.x; r = r && a.lo.y <= b.lo.y;
    r = r && b.hi.x <= a.hi.x; r = r && b.hi.y <= a.hi.y;
    return r;
}

/* ---- body helpers (b2Body) ---- */
static void set_awake(oworld *w) { if (!w->awake) { w->awake = 1; w->sleepTime = 0.0f; } }
static void sync_transform(oworld *w) {
    ob_rot_set(&w->xf.q, w->a);
    w->xf.p = vsub(w->c, rmul(w->xf.q, V(0.0f, 0.0f)));
}
void ob_apply_force(oworld *w, ov2 f, ov2 point) {
    set_awake(w);
    w->force = vadd(w->force, f);
    w->torque += vcross(vsub(point, w->c), f);
}
void ob_apply_force_center(oworld *w, ov2 f) { set_awake(w); w->force = vadd(w->force, f); }
void ob_apply_torque(oworld *w, float t) { set_awake(w); w->torque += t; }

/* b2Fixture::Synchronize + b2DynamicTree::MoveProxy for the car proxy */
static void move_proxy(oworld *w, oxf xf1, oxf xf2) {
    opoly cp; car_poly(&cp);
    oaabb a1 = poly_aabb(&cp, xf1), a2 = poly_aabb(&cp, xf2), aabb;
    aabb.lo = vmin(a1.lo, a2.lo); aabb.hi = vmax(a1.hi, a2.hi);
    ov2 disp = vsub(xf2.p, xf1.p);
    if (contains(w->fat, aabb)) return;
    oaabb b = aabb; ov2 r = V(AABB_EXT, AABB_EXT);
    b.lo = vsub(b.lo, r); b.hi = vadd(b.hi, r);
    ov2 d = vmul(AABB_MULT, disp);
    if (d.x < 0.0f) b.lo.x += d.x; else b.hi.x += d.x;
    if (d.y < 0.0f) b.lo.y += d.y; else b.hi.y += d.y;
    w->fat = b; w->moved = 1;
}
/* b2Body::SynchronizeFixtures */
static void sync_fixtures(oworld *w) {
    oxf xf1; ob_rot_set(&xf1.q, w->a0);
    xf1.p = vsub(w->c0, rmul(xf1.q, V(0.0f, 0.0f)));
    move_proxy(w, xf1, w->xf);
}

/* ---- contacts / broadphase pairs (b2ContactManager) ---- */
static int find_contact(const oworld *w, int wall) {
    for (int i = 0; i < w->nct; ++i) if (w->ct[i].wall == wall) return i;
    return -1;
}
/* b2BroadPhase::UpdatePairs: pairs sorted by (proxyIdA, proxyIdB); the car proxy
 * is 0 and wall proxy ids grow with wall creation order, so AddPair runs in
 * ascending wall index and each new contact is prepended to the lists. */
static void find_new_contacts(oworld *w, const owalls *W) {
    if (!w->moved) return;
    w->moved = 0;
    for (int j = 0; j < W->n; ++j) {
        if (!overlap(w->fat, W->fat[j])) continue;
        if (find_contact(w, j) >= 0) continue;
        if (w->nct >= OB_MAXC) { w->overflow = 1; continue; }
        memmove(&w->ct[1], &w->ct[0], sizeof(ocontact) * (size_t)w->nct);
        ocontact *c = &w->ct[0];
        memset(c, 0, sizeof(*c));
        c->wall = j; c->flags = OC_ENABLED; c->toi = 1.0f;
        w->nct++;
        set_awake(w);
    }
}
static void remove_contact(oworld *w, int i) {
    memmove(&w->ct[i], &w->ct[i + 1], sizeof(ocontact) * (size_t)(w->nct - i - 1));
    w->nct--;
}

/* ---- b2CollidePolygons (Box2D 2.3.1+) ---- */
typedef struct { ov2 v; uint32_t id; } oclip;
static inline uint32_t cf_key(int ia, int ib, int ta, int tb) {
    return (uint32_t)(ia & 255) | ((uint32_t)(ib & 255) << 8) | ((uint32_t)(ta & 255) << 16) | ((uint32_t)(tb & 255) << 24);
}
static float find_max_separation(int *edgeIndex, const opoly *p1, oxf xf1, const opoly *p2, oxf xf2) {
    oxf xf = xmulT_xx(xf2, xf1);
    int best = 0; float maxSep = -FLT_MAX;
    for (int i = 0; i < p1->count; ++i) {
        ov2 n = rmul(xf.q, p1->n[i]);
        ov2 v1 = xmul(xf, p1->v[i]);
        float si = FLT_MAX;
        for (int j = 0; j < p2->count; ++j) {
            float sij = vdot(n, vsub(p2->v[j], v1));
            if (sij < si) si = sij;
        }
        if (si > maxSep) { maxSep = si; best = i; }
    }
    *edgeIndex = best;
    return maxSep;
}
static void find_incident_edge(oclip c[2], const opoly *p1, oxf xf1, int edge1, const opoly *p2, oxf xf2) {
    ov2 normal1 = rmulT(xf2.q, rmul(xf1.q, p1->n[edge1]));
    int index = 0; float minDot = FLT_MAX;
    for (int i = 0; i < p2->count; ++i) {
        float d = vdot(normal1, p2->n[i]);
        if (d < minDot) { minDot = d; index = i; }
    }
    int i1 = index, i2 = i1 + 1 < p2->count ? i1 + 1 : 0;
    c[0].v = xmul(xf2, p2->v[i1]); c[0].id = cf_key(edge1, i1, 1, 0);
    c[1].v = xmul(xf2, p2->v[i2]); c[1].id = cf_key(edge1, i2, 1, 0);
}
static int clip_segment(oclip vOut[2], const oclip vIn[2], ov2 normal, float offset, int vertexIndexA) {
    int numOut = 0;
    float d0 = vdot(normal, vIn[0].v) - offset;
    float d1 = vdot(normal, vIn[1].v) - offset;
    if (d0 <= 0.0f) vOut[numOut++] = vIn[0];
    if (d1 <= 0.0f) vOut[numOut++] = vIn[1];
    if (d0 * d1 < 0.0f) {
        float interp = d0 / (d0 - d1);
        vOut[numOut].v = vadd(vIn[0].v, vmul(interp, vsub(vIn[1].v, vIn[0].v)));
        vOut[numOut].id = cf_key(vertexIndexA, (int)((vIn[0].id >> 8) & 255), 0, 1);
        ++numOut;
    }
    return numOut;
}
static void collide_polygons(omanifold *m, const opoly *pA, oxf xfA, const opoly *pB, oxf xfB) {
    m->pointCount = 0;
    float totalRadius = pA->radius + pB->radius;
    int edgeA = 0; float sepA = find_max_separation(&edgeA, pA, xfA, pB, xfB);
    if (sepA > totalRadius) return;
    int edgeB = 0; float sepB = find_max_separation(&edgeB, pB, xfB, pA, xfA);
    if (sepB > totalRadius) return;
    const opoly *poly1, *poly2; oxf xf1, xf2; int edge1; int flip;
    const float k_tol = 0.1f * LINEAR_SLOP;
    if (sepB > sepA + k_tol) { poly1 = pB; poly2 = pA; xf1 = xfB; xf2 = xfA; edge1 = edgeB; m->type = 2; flip = 1; }
    else { poly1 = pA; poly2 = pB; xf1 = xfA; xf2 = xfB; edge1 = edgeA; m->type = 1; flip = 0; }
    oclip incident[2];
    find_incident_edge(incident, poly1, xf1, edge1, poly2, xf2);
    int count1 = poly1->count;
    int iv1 = edge1, iv2 = edge1 + 1 < count1 ? edge1 + 1 : 0;
    ov2 v11 = poly1->v[iv1], v12 = poly1->v[iv2];
    ov2 localTangent = vsub(v12, v11);
    vnormalize(&localTangent);
    ov2 localNormal = vcross_vs(localTangent, 1.0f);
    ov2 planePoint = vmul(0.5f, vadd(v11, v12));
    ov2 tangent = rmul(xf1.q, localTangent);
    ov2 normal = vcross_vs(tangent, 1.0f);
    v11 = xmul(xf1, v11); v12 = xmul(xf1, v12);
    float frontOffset = vdot(normal, v11);
    float sideOffset1 = -vdot(tangent, v11) + totalRadius;
    float sideOffset2 = vdot(tangent, v12) + totalRadius;
    oclip cp1[2], cp2[2];
    int np = clip_segment(cp1, incident, vneg(tangent), sideOffset1, iv1);
    if (np < 2) return;
    np = clip_segment(cp2, cp1, tangent, sideOffset2, iv2);
    if (np < 2) return;
    m->localNormal = localNormal; m->localPoint = planePoint;
    int pc = 0;
    for (int i = 0; i < 2; ++i) {
        float separation = vdot(normal, cp2[i].v) - frontOffset;
        if (separation <= totalRadius) {
            ompt *p = &m->pts[pc];
            p->localPoint = xmulT(xf2, cp2[i].v);
            uint32_t id = cp2[i].id;
            if (flip) {
                uint32_t ia = id & 255, ib = (id >> 8) & 255, ta = (id >> 16) & 255, tb = (id >> 24) & 255;
                id = cf_key((int)ib, (int)ia, (int)tb, (int)ta);
            }
            p->id = id; p->normalImpulse = 0.0f; p->tangentImpulse = 0.0f;
            ++pc;
        }
    }
    m->pointCount = pc;
}

/* b2WorldManifold::Initialize (face manifolds only) */
static void world_manifold(const omanifold *m, oxf xfA, float rA, oxf xfB, float rB, ov2 *normal, ov2 pts[2]) {
    if (m->pointCount == 0) return;
    if (m->type == 1) {
        ov2 n = rmul(xfA.q, m->localNormal);
        ov2 planePoint = xmul(xfA, m->localPoint);
        for (int i = 0; i < m->pointCount; ++i) {
            ov2 clipPoint = xmul(xfB, m->pts[i].localPoint);
            ov2 cA = vadd(clipPoint, vmul(rA - vdot(vsub(clipPoint, planePoint), n), n));
            ov2 cB = vsub(clipPoint, vmul(rB, n));
            pts[i] = vmul(0.5f, vadd(cA, cB));
        }
        *normal = n;
    } else {
        ov2 n = rmul(xfB.q, m->localNormal);
        ov2 planePoint = xmul(xfB, m->localPoint);
        for (int i = 0; i < m->pointCount; ++i) {
            ov2 clipPoint = xmul(xfA, m->pts[i].localPoint);
            ov2 cB = vadd(clipPoint, vmul(rB - vdot(vsub(clipPoint, planePoint), n), n));
            ov2 cA = vsub(clipPoint, vmul(rA, n));
            pts[i] = vmul(0.5f, vadd(cA, cB));
        }
        *normal = vneg(n);
    }
}

/* b2Contact::Update (polygon-polygon, no sensors) */
static void contact_update(oworld *w, int ci, const owalls *W, const olistener *L) {
    ocontact *c = &w->ct[ci];
    omanifold old = c->m;
    c->flags |= OC_ENABLED;
    int was = (c->flags & OC_TOUCH) != 0;
    opoly pa, pb; car_poly(&pa); wall_poly(&pb, W, c->wall);
    oxf xfB = wall_xf(W, c->wall);
    collide_polygons(&c->m, &pa, w->xf, &pb, xfB);
    int touching = c->m.pointCount > 0;
    for (int i = 0; i < c->m.pointCount; ++i) {
        ompt *p2 = &c->m.pts[i];
        p2->normalImpulse = 0.0f; p2->tangentImpulse = 0.0f;
        for (int j = 0; j < old.pointCount; ++j) {
            if (old.pts[j].id == p2->id) {
                p2->normalImpulse = old.pts[j].normalImpulse;
                p2->tangentImpulse = old.pts[j].tangentImpulse;
                break;
            }
        }
    }
    if (touching != was) set_awake(w);
    if (touching) c->flags |= OC_TOUCH; else c->flags &= ~OC_TOUCH;
    if (!was && touching && L && L->begin) {
        ov2 n = V(0, 0), pts[2];
        world_manifold(&c->m, w->xf, POLY_RADIUS, xfB, POLY_RADIUS, &n, pts);
        L->begin(L->user, c->wall, n);
    }
    if (was && !touching && L && L->end) L->end(L->user, c->wall);
}

/* b2ContactManager::Collide */
static void collide(oworld *w, const owalls *W, const olistener *L) {
    int i = 0;
    while (i < w->nct) {
        ocontact *c = &w->ct[i];
        if (!w->awake) { ++i; continue; }
        if (!overlap(w->fat, W->fat[c->wall])) {
            int touching = (c->flags & OC_TOUCH) != 0, wall = c->wall;
            remove_contact(w, i);
            if (touching && L && L->end) L->end(L->user, wall);
            continue;
        }
        contact_update(w, i, W, L);
        ++i;
    }
}

/* ---- b2ContactSolver ---- */
typedef struct {
    ov2 rA, rB; float normalImpulse, tangentImpulse, normalMass, tangentMass, velocityBias;
} ovcp;
typedef struct {
    ovcp pts[2]; ov2 normal; float nm[4] /* normalMass ex.x, ex.y, ey.x, ey.y */; float K[4];
    int pointCount; float friction, restitution;
    /* wall body (static): index-B state */
    ov2 cB; float aB; ov2 vB; float wB;
    /* position constraint */
    ov2 localNormal, localPoint, localPoints[2]; int pcount; int type;
    int ci; int wall;
} ovc;

typedef struct { ov2 c; float a; ov2 v; float w; } obodystate;

static void cs_init(ovc *vc, int n, const oworld *w, const int *cidx, const owalls *W, int warm, float dtRatio) {
    for (int i = 0; i < n; ++i) {
        const ocontact *c = &w->ct[cidx[i]];
        ovc *v = &vc[i];
        memset(v, 0, sizeof(*v));
        v->ci = cidx[i]; v->wall = c->wall;
        v->friction = mix_friction(); v->restitution = MIX_RESTITUTION;
        v->pointCount = c->m.pointCount;
        v->cB = W->p[c->wall]; v->aB = W->angle[c->wall]; v->vB = V(0.0f, 0.0f); v->wB = 0.0f;
        v->localNormal = c->m.localNormal; v->localPoint = c->m.localPoint; v->pcount = c->m.pointCount; v->type = c->m.type;
        for (int j = 0; j < c->m.pointCount; ++j) {
            const ompt *cp = &c->m.pts[j];
            ovcp *p = &v->pts[j];
            if (warm) { p->normalImpulse = dtRatio * cp->normalImpulse; p->tangentImpulse = dtRatio * cp->tangentImpulse; }
            else { p->normalImpulse = 0.0f; p->tangentImpulse = 0.0f; }
            v->localPoints[j] = cp->localPoint;
        }
    }
}

static void cs_init_velocity(ovc *vc, int n, const oworld *w, const obodystate *A) {
    const float mA = CAR_INV_MASS, iA = CAR_INV_I, mB = 0.0f, iB = 0.0f;
    for (int i = 0; i < n; ++i) {
        ovc *v = &vc[i];
        const omanifold *m = &w->ct[v->ci].m;
        ov2 cA = A->c; float aA = A->a; ov2 vA = A->v; float wA = A->w;
        ov2 cB = v->cB; float aB = v->aB; ov2 vB = v->vB; float wB = v->wB;
        oxf xfA, xfB;
        ob_rot_set(&xfA.q, aA); ob_rot_set(&xfB.q, aB);
        xfA.p = vsub(cA, rmul(xfA.q, V(0.0f, 0.0f)));
        xfB.p = vsub(cB, rmul(xfB.q, V(0.0f, 0.0f)));
        ov2 normal = V(0, 0), pts[2];
        world_manifold(m, xfA, POLY_RADIUS, xfB, POLY_RADIUS, &normal, pts);
        v->normal = normal;
        for (int j = 0; j < v->pointCount; ++j) {
            ovcp *p = &v->pts[j];
            p->rA = vsub(pts[j], cA); p->rB = vsub(pts[j], cB);
            float rnA = vcross(p->rA, v->normal), rnB = vcross(p->rB, v->normal);
            float kNormal = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
            p->normalMass = kNormal > 0.0f ? 1.0f / kNormal : 0.0f;
            ov2 tangent = vcross_vs(v->normal, 1.0f);
            float rtA = vcross(p->rA, tangent), rtB = vcross(p->rB, tangent);
            float kTangent = mA + mB + iA * rtA * rtA + iB * rtB * rtB;
            p->tangentMass = kTangent > 0.0f ? 1.0f / kTangent : 0.0f;
            p->velocityBias = 0.0f;
            float vRel = vdot(v->normal, vsub(vsub(vadd(vB, vcross_sv(wB, p->rB)), vA), vcross_sv(wA, p->rA)));
            if (vRel < -VELOCITY_THRESHOLD) p->velocityBias = -v->restitution * vRel;
        }
        if (v->pointCount == 2) {
            ovcp *p1 = &v->pts[0], *p2 = &v->pts[1];
            float rn1A = vcross(p1->rA, v->normal), rn1B = vcross(p1->rB, v->normal);
            float rn2A = vcross(p2->rA, v->normal), rn2B = vcross(p2->rB, v->normal);
            float k11 = mA + mB + iA * rn1A * rn1A + iB * rn1B * rn1B;
            float k22 = mA + mB + iA * rn2A * rn2A + iB * rn2B * rn2B;
            float k12 = mA + mB + iA * rn1A * rn2A + iB * rn1B * rn2B;
            const float k_maxConditionNumber = 1000.0f;
            if (k11 * k11 < k_maxConditionNumber * (k11 * k22 - k12 * k12)) {
                v->K[0] = k11; v->K[1] = k12; v->K[2] = k12; v->K[3] = k22;   /* ex=(k11,k12) ey=(k12,k22) */
                float a = v->K[0], b = v->K[2], cc = v->K[1], d = v->K[3];
                float det = a * d - b * cc;
                if (det != 0.0f) det = 1.0f / det;
                v->nm[0] = det * d; v->nm[2] = -det * b; v->nm[1] = -det * cc; v->nm[3] = det * a;
            } else {
                v->pointCount = 1;
            }
        }
    }
}

static void cs_warm_start(ovc *vc, int n, obodystate *A) {
    const float mA = CAR_INV_MASS, iA = CAR_INV_I, mB = 0.0f, iB = 0.0f;
    for (int i = 0; i < n; ++i) {
        ovc *v = &vc[i];
        ov2 vA = A->v; float wA = A->w; ov2 vB = v->vB; float wB = v->wB;
        ov2 normal = v->normal, tangent = vcross_vs(normal, 1.0f);
        for (int j = 0; j < v->pointCount; ++j) {
            ovcp *p = &v->pts[j];
            ov2 P = vadd(vmul(p->normalImpulse, normal), vmul(p->tangentImpulse, tangent));
            wA -= iA * vcross(p->rA, P);
            vA = vsub(vA, vmul(mA, P));
            wB += iB * vcross(p->rB, P);
            vB = vadd(vB, vmul(mB, P));
        }
        A->v = vA; A->w = wA; v->vB = vB; v->wB = wB;
    }
}

static inline ov2 rel_vel(ov2 vA, float wA, ov2 vB, float wB, const ovcp *p) {
    return vsub(vsub(vadd(vB, vcross_sv(wB, p->rB)), vA), vcross_sv(wA, p->rA));
}

static void cs_solve_velocity(ovc *vc, int n, obodystate *A) {
    const float mA = CAR_INV_MASS, iA = CAR_INV_I, mB = 0.0f, iB = 0.0f;
    for (int i = 0; i < n; ++i) {
        ovc *v = &vc[i];
        ov2 vA = A->v; float wA = A->w; ov2 vB = v->vB; float wB = v->wB;
        ov2 normal = v->normal, tangent = vcross_vs(normal, 1.0f);
        float friction = v->friction;
        for (int j = 0; j < v->pointCount; ++j) {
            ovcp *p = &v->pts[j];
            ov2 dv = rel_vel(vA, wA, vB, wB, p);
            float vt = vdot(dv, tangent) - 0.0f;
            float lambda = p->tangentMass * (-vt);
            float maxFriction = friction * p->normalImpulse;
            float newImpulse = fclamp(p->tangentImpulse + lambda, -maxFriction, maxFriction);
            lambda = newImpulse - p->tangentImpulse;
            p->tangentImpulse = newImpulse;
            ov2 P = vmul(lambda, tangent);
            vA = vsub(vA, vmul(mA, P)); wA -= iA * vcross(p->rA, P);
            vB = vadd(vB, vmul(mB, P)); wB += iB * vcross(p->rB, P);
        }
        if (v->pointCount == 1) {
            ovcp *p = &v->pts[0];
            ov2 dv = rel_vel(vA, wA, vB, wB, p);
            float vn = vdot(dv, normal);
            float lambda = -p->normalMass * (vn - p->velocityBias);
            float newImpulse = fmax_b2(p->normalImpulse + lambda, 0.0f);
            lambda = newImpulse - p->normalImpulse;
            p->normalImpulse = newImpulse;
            ov2 P = vmul(lambda, normal);
            vA = vsub(vA, vmul(mA, P)); wA -= iA * vcross(p->rA, P);
            vB = vadd(vB, vmul(mB, P)); wB += iB * vcross(p->rB, P);
        } else {
            ovcp *cp1 = &v->pts[0], *cp2 = &v->pts[1];
            ov2 a = V(cp1->normalImpulse, cp2->normalImpulse);
            ov2 dv1 = rel_vel(vA, wA, vB, wB, cp1), dv2 = rel_vel(vA, wA, vB, wB, cp2);
            float vn1 = vdot(dv1, normal), vn2 = vdot(dv2, normal);
            ov2 b = V(vn1 - cp1->velocityBias, vn2 - cp2->velocityBias);
            /* b -= K * a  (b2Mul(Mat22, v) = (ex.x*v.x + ey.x*v.y, ex.y*v.x + ey.y*v.y)) */
            ov2 Ka = V(v->K[0] * a.x + v->K[2] * a.y, v->K[1] * a.x + v->K[3] * a.y);
            b = vsub(b, Ka);
            for (;;) {
                ov2 x = vneg(V(v->nm[0] * b.x + v->nm[2] * b.y, v->nm[1] * b.x + v->nm[3] * b.y));
                if (x.x >= 0.0f && x.y >= 0.0f) goto apply;
                x.x = -cp1->normalMass * b.x; x.y = 0.0f;
                vn1 = 0.0f; vn2 = v->K[1] * x.x + b.y;
                if (x.x >= 0.0f && vn2 >= 0.0f) goto apply;
                x.x = 0.0f; x.y = -cp2->normalMass * b.y;
                vn1 = v->K[2] * x.y + b.x; vn2 = 0.0f;
                if (x.y >= 0.0f && vn1 >= 0.0f) goto apply;
                x.x = 0.0f; x.y = 0.0f; vn1 = b.x; vn2 = b.y;
                if (vn1 >= 0.0f && vn2 >= 0.0f) goto apply;
                break;
            apply: {
                    ov2 d = vsub(x, a);
                    ov2 P1 = vmul(d.x, normal), P2 = vmul(d.y, normal);
                    vA = vsub(vA, vmul(mA, vadd(P1, P2)));
                    wA -= iA * (vcross(cp1->rA, P1) + vcross(cp2->rA, P2));
                    vB = vadd(vB, vmul(mB, vadd(P1, P2)));
                    wB += iB * (vcross(cp1->rB, P1) + vcross(cp2->rB, P2));
                    cp1->normalImpulse = x.x; cp2->normalImpulse = x.y;
                    break;
                }
            }
        }
        A->v = vA; A->w = wA; v->vB = vB; v->wB = wB;
    }
}

static void cs_store(const ovc *vc, int n, oworld *w) {
    for (int i = 0; i < n; ++i) {
        omanifold *m = &w->ct[vc[i].ci].m;
        for (int j = 0; j < vc[i].pointCount; ++j) {
            m->pts[j].normalImpulse = vc[i].pts[j].normalImpulse;
            m->pts[j].tangentImpulse = vc[i].pts[j].tangentImpulse;
        }
    }
}

/* b2PositionSolverManifold::Initialize */
static void psm(const ovc *v, oxf xfA, oxf xfB, int idx, ov2 *normal, ov2 *point, float *sep) {
    if (v->type == 1) {
        ov2 n = rmul(xfA.q, v->localNormal);
        ov2 planePoint = xmul(xfA, v->localPoint);
        ov2 clipPoint = xmul(xfB, v->localPoints[idx]);
        *sep = vdot(vsub(clipPoint, planePoint), n) - POLY_RADIUS - POLY_RADIUS;
        *point = clipPoint; *normal = n;
    } else {
        ov2 n = rmul(xfB.q, v->localNormal);
        ov2 planePoint = xmul(xfB, v->localPoint);
        ov2 clipPoint = xmul(xfA, v->localPoints[idx]);
        *sep = vdot(vsub(clipPoint, planePoint), n) - POLY_RADIUS - POLY_RADIUS;
        *point = clipPoint; *normal = vneg(n);
    }
}

/* SolvePositionConstraints (toi=0) / SolveTOIPositionConstraints (toi=1) */
static int cs_solve_position(ovc *vc, int n, obodystate *A, int toi) {
    float minSep = 0.0f;
    const float mA = CAR_INV_MASS, iA = CAR_INV_I, mB = 0.0f, iB = 0.0f;
    for (int i = 0; i < n; ++i) {
        ovc *v = &vc[i];
        ov2 cA = A->c; float aA = A->a; ov2 cB = v->cB; float aB = v->aB;
        for (int j = 0; j < v->pcount; ++j) {
            oxf xfA, xfB;
            ob_rot_set(&xfA.q, aA); ob_rot_set(&xfB.q, aB);
            xfA.p = vsub(cA, rmul(xfA.q, V(0.0f, 0.0f)));
            xfB.p = vsub(cB, rmul(xfB.q, V(0.0f, 0.0f)));
            ov2 normal, point; float sep;
            psm(v, xfA, xfB, j, &normal, &point, &sep);
            ov2 rA = vsub(point, cA), rB = vsub(point, cB);
            minSep = fmin_b2(minSep, sep);
            float C = fclamp((toi ? TOI_BAUMGARTE : BAUMGARTE) * (sep + LINEAR_SLOP), -MAX_LINEAR_CORRECTION, 0.0f);
            float rnA = vcross(rA, normal), rnB = vcross(rB, normal);
            float K = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
            float impulse = K > 0.0f ? -C / K : 0.0f;
            ov2 P = vmul(impulse, normal);
            cA = vsub(cA, vmul(mA, P)); aA -= iA * vcross(rA, P);
            cB = vadd(cB, vmul(mB, P)); aB += iB * vcross(rB, P);
        }
        A->c = cA; A->a = aA; v->cB = cB; v->aB = aB;
    }
    return toi ? (minSep >= -1.5f * LINEAR_SLOP) : (minSep >= -3.0f * LINEAR_SLOP);
}

static void report(const ovc *vc, int n, const olistener *L) {
    if (!L || !L->post) return;
    for (int i = 0; i < n; ++i) {
        float ni[2] = { vc[i].pts[0].normalImpulse, vc[i].pts[1].normalImpulse };
        L->post(L->user, vc[i].pointCount, ni);
    }
}

/* integrate positions with the b2_maxTranslation / b2_maxRotation clamps */
static void integrate_positions(obodystate *A, float h) {
    ov2 c = A->c; float a = A->a; ov2 v = A->v; float w = A->w;
    ov2 translation = vmul(h, v);
    if (vdot(translation, translation) > MAX_TRANSLATION_SQ) {
        float ratio = MAX_TRANSLATION / vlen(translation);
        v = vmul(ratio, v);
    }
    float rotation = h * w;
    if (rotation * rotation > MAX_ROTATION_SQ) {
        float ratio = MAX_ROTATION / fabsf(rotation);
        w *= ratio;
    }
    c = vadd(c, vmul(h, v));
    a += h * w;
    A->c = c; A->a = a; A->v = v; A->w = w;
}

/* b2World::Solve with the single-dynamic-body island of this world (b2Island::Solve) */
static void solve(oworld *w, const owalls *W, const olistener *L, float dt, float dtRatio, int velIters, int posIters) {
    if (!w->awake) return;           /* seed must be awake; nothing else moves */
    int cidx[OB_MAXC], n = 0;
    for (int i = 0; i < w->nct; ++i) {
        const ocontact *c = &w->ct[i];
        if (!(c->flags & OC_ENABLED) || !(c->flags & OC_TOUCH)) continue;
        cidx[n++] = i;
    }
    float h = dt;
    obodystate A;
    w->c0 = w->c; w->a0 = w->a;
    {
        ov2 v = w->v; float wv = w->w;
        ov2 g = vadd(vmul(1.0f, V(0.0f, 0.0f)), vmul(CAR_INV_MASS, w->force));
        v = vadd(v, vmul(h, g));
        wv += h * CAR_INV_I * w->torque;
        A.c = w->c; A.a = w->a; A.v = v; A.w = wv;
    }
    ovc vc[OB_MAXC];
    cs_init(vc, n, w, cidx, W, 1, dtRatio);
    cs_init_velocity(vc, n, w, &A);
    cs_warm_start(vc, n, &A);
    for (int it = 0; it < velIters; ++it) cs_solve_velocity(vc, n, &A);
    cs_store(vc, n, w);
    integrate_positions(&A, h);
    int positionSolved = 0;
    for (int it = 0; it < posIters; ++it) {
        if (cs_solve_position(vc, n, &A, 0)) { positionSolved = 1; break; }
    }
    w->c = A.c; w->a = A.a; w->v = A.v; w->w = A.w;
    sync_transform(w);
    report(vc, n, L);
    /* sleep */
    {
        float minSleepTime = FLT_MAX;
        const float linTolSqr = LINEAR_SLEEP_TOL * LINEAR_SLEEP_TOL;
        const float angTolSqr = ANGULAR_SLEEP_TOL * ANGULAR_SLEEP_TOL;
        if (w->w * w->w > angTolSqr || vdot(w->v, w->v) > linTolSqr) { w->sleepTime = 0.0f; minSleepTime = 0.0f; }
        else { w->sleepTime += h; minSleepTime = fmin_b2(minSleepTime, w->sleepTime); }
        if (minSleepTime >= TIME_TO_SLEEP && positionSolved) {
            w->awake = 0; w->sleepTime = 0.0f; w->v = V(0.0f, 0.0f); w->w = 0.0f;
            w->force = V(0.0f, 0.0f); w->torque = 0.0f;
        }
    }
    /* synchronize fixtures of the (island) car, then look for new contacts */
    sync_fixtures(w);
    find_new_contacts(w, W);
}

/* ---- b2Distance (GJK) ---- */
typedef struct { ov2 wA, wB, w; float a; int indexA, indexB; } osv;
typedef struct { osv v[3]; int count; } osimplex;
typedef struct { float metric; int count; int indexA[3], indexB[3]; } ocache;

static int support(const opoly *p, ov2 d) {
    int best = 0; float bestValue = vdot(p->v[0], d);
    for (int i = 1; i < p->count; ++i) { float value = vdot(p->v[i], d); if (value > bestValue) { best = i; bestValue = value; } }
    return best;
}
static float simplex_metric(const osimplex *s) {
    switch (s->count) {
    case 1: return 0.0f;
    case 2: return vlen(vsub(s->v[0].w, s->v[1].w));
    case 3: return vcross(vsub(s->v[1].w, s->v[0].w), vsub(s->v[2].w, s->v[0].w));
    default: return 0.0f;
    }
}
static void read_cache(osimplex *s, const ocache *cache, const opoly *pA, oxf tA, const opoly *pB, oxf tB) {
    s->count = cache->count;
    for (int i = 0; i < s->count; ++i) {
        osv *v = &s->v[i];
        v->indexA = cache->indexA[i]; v->indexB = cache->indexB[i];
        v->wA = xmul(tA, pA->v[v->indexA]); v->wB = xmul(tB, pB->v[v->indexB]);
        v->w = vsub(v->wB, v->wA); v->a = 0.0f;
    }
    if (s->count > 1) {
        float metric1 = cache->metric, metric2 = simplex_metric(s);
        if (metric2 < 0.5f * metric1 || 2.0f * metric1 < metric2 || metric2 < FLT_EPSILON) s->count = 0;
    }
    if (s->count == 0) {
        osv *v = &s->v[0];
        v->indexA = 0; v->indexB = 0;
        v->wA = xmul(tA, pA->v[0]); v->wB = xmul(tB, pB->v[0]);
        v->w = vsub(v->wB, v->wA); v->a = 1.0f;
        s->count = 1;
    }
}
static void write_cache(const osimplex *s, ocache *cache) {
    cache->metric = simplex_metric(s);
    cache->count = s->count;
    for (int i = 0; i < s->count; ++i) { cache->indexA[i] = s->v[i].indexA; cache->indexB[i] = s->v[i].indexB; }
}
static ov2 search_direction(const osimplex *s) {
    if (s->count == 1) return vneg(s->v[0].w);
    ov2 e12 = vsub(s->v[1].w, s->v[0].w);
    float sgn = vcross(e12, vneg(s->v[0].w));
    if (sgn > 0.0f) return vcross_sv(1.0f, e12);
    return vcross_vs(e12, 1.0f);
}
static ov2 closest_point(const osimplex *s) {
    switch (s->count) {
    case 1: return s->v[0].w;
    case 2: return vadd(vmul(s->v[0].a, s->v[0].w), vmul(s->v[1].a, s->v[1].w));
    default: return V(0.0f, 0.0f);
    }
}
static void witness(const osimplex *s, ov2 *pA, ov2 *pB) {
    switch (s->count) {
    case 1: *pA = s->v[0].wA; *pB = s->v[0].wB; break;
    case 2:
        *pA = vadd(vmul(s->v[0].a, s->v[0].wA), vmul(s->v[1].a, s->v[1].wA));
        *pB = vadd(vmul(s->v[0].a, s->v[0].wB), vmul(s->v[1].a, s->v[1].wB));
        break;
    case 3:
        *pA = vadd(vadd(vmul(s->v[0].a, s->v[0].wA), vmul(s->v[1].a, s->v[1].wA)), vmul(s->v[2].a, s->v[2].wA));
        *pB = *pA;
        break;
    default: break;
    }
}
static void solve2(osimplex *s) {
    ov2 w1 = s->v[0].w, w2 = s->v[1].w, e12 = vsub(w2, w1);
    float d12_2 = -vdot(w1, e12);
    if (d12_2 <= 0.0f) { s->v[0].a = 1.0f; s->count = 1; return; }
    float d12_1 = vdot(w2, e12);
    if (d12_1 <= 0.0f) { s->v[1].a = 1.0f; s->count = 1; s->v[0] = s->v[1]; return; }
    float inv = 1.0f / (d12_1 + d12_2);
    s->v[0].a = d12_1 * inv; s->v[1].a = d12_2 * inv; s->count = 2;
}
static void solve3(osimplex *s) {
    ov2 w1 = s->v[0].w, w2 = s->v[1].w, w3 = s->v[2].w;
    ov2 e12 = vsub(w2, w1);
    float w1e12 = vdot(w1, e12), w2e12 = vdot(w2, e12);
    float d12_1 = w2e12, d12_2 = -w1e12;
    ov2 e13 = vsub(w3, w1);
    float w1e13 = vdot(w1, e13), w3e13 = vdot(w3, e13);
    float d13_1 = w3e13, d13_2 = -w1e13;
    ov2 e23 = vsub(w3, w2);
    float w2e23 = vdot(w2, e23), w3e23 = vdot(w3, e23);
    float d23_1 = w3e23, d23_2 = -w2e23;
    float n123 = vcross(e12, e13);
    float d123_1 = n123 * vcross(w2, w3);
    float d123_2 = n123 * vcross(w3, w1);
    float d123_3 = n123 * vcross(w1, w2);
    if (d12_2 <= 0.0f && d13_2 <= 0.0f) { s->v[0].a = 1.0f; s->count = 1; return; }
    if (d12_1 > 0.0f && d12_2 > 0.0f && d123_3 <= 0.0f) {
        float inv = 1.0f / (d12_1 + d12_2); s->v[0].a = d12_1 * inv; s->v[1].a = d12_2 * inv; s->count = 2; return;
    }
    if (d13_1 > 0.0f && d13_2 > 0.0f && d123_2 <= 0.0f) {
        float inv = 1.0f / (d13_1 + d13_2); s->v[0].a = d13_1 * inv; s->v[2].a = d13_2 * inv; s->count = 2; s->v[1] = s->v[2]; return;
    }
    if (d12_1 <= 0.0f && d23_2 <= 0.0f) { s->v[1].a = 1.0f; s->count = 1; s->v[0] = s->v[1]; return; }
    if (d13_1 <= 0.0f && d23_1 <= 0.0f) { s->v[2].a = 1.0f; s->count = 1; s->v[0] = s->v[2]; return; }
    if (d23_1 > 0.0f && d23_2 > 0.0f && d123_1 <= 0.0f) {
        float inv = 1.0f / (d23_1 + d23_2); s->v[1].a = d23_1 * inv; s->v[2].a = d23_2 * inv; s->count = 2; s->v[0] = s->v[2]; return;
    }
    float inv = 1.0f / (d123_1 + d123_2 + d123_3);
    s->v[0].a = d123_1 * inv; s->v[1].a = d123_2 * inv; s->v[2].a = d123_3 * inv; s->count = 3;
}
static float gjk_distance(ocache *cache, const opoly *pA, oxf tA, const opoly *pB, oxf tB) {
    osimplex s;
    read_cache(&s, cache, pA, tA, pB, tB);
    int saveA[3], saveB[3], saveCount = 0, iter = 0;
    while (iter < 20) {
        saveCount = s.count;
        for (int i = 0; i < saveCount; ++i) { saveA[i] = s.v[i].indexA; saveB[i] = s.v[i].indexB; }
        if (s.count == 2) solve2(&s); else if (s.count == 3) solve3(&s);
        if (s.count == 3) break;
        ov2 p = closest_point(&s); (void)p;
        ov2 d = search_direction(&s);
        if (vdot(d, d) < FLT_EPSILON * FLT_EPSILON) break;
        osv *vx = &s.v[s.count];
        vx->indexA = support(pA, rmulT(tA.q, vneg(d)));
        vx->wA = xmul(tA, pA->v[vx->indexA]);
        vx->indexB = support(pB, rmulT(tB.q, d));
        vx->wB = xmul(tB, pB->v[vx->indexB]);
        vx->w = vsub(vx->wB, vx->wA);
        ++iter;
        int dup = 0;
        for (int i = 0; i < saveCount; ++i) if (vx->indexA == saveA[i] && vx->indexB == saveB[i]) { dup = 1; break; }
        if (dup) break;
        ++s.count;
    }
    ov2 wa = V(0, 0), wb = V(0, 0);
    witness(&s, &wa, &wb);
    write_cache(&s, cache);
    return vlen(vsub(wa, wb));
}

/* ---- b2TimeOfImpact ---- */
typedef struct { ov2 c0, c; float a0, a, alpha0; } osweep;   /* localCenter == (0,0) for every body here */
static oxf sweep_xf(const osweep *s, float beta) {
    oxf xf;
    xf.p = vadd(vmul(1.0f - beta, s->c0), vmul(beta, s->c));
    float angle = (1.0f - beta) * s->a0 + beta * s->a;
    ob_rot_set(&xf.q, angle);
    xf.p = vsub(xf.p, rmul(xf.q, V(0.0f, 0.0f)));
    return xf;
}
static void sweep_normalize(osweep *s) {
    float twoPi = 2.0f * B2_PI;
    float d = twoPi * floorf(s->a0 / twoPi);
    s->a0 -= d; s->a -= d;
}
static void sweep_advance(osweep *s, float alpha) {
    float beta = (alpha - s->alpha0) / (1.0f - s->alpha0);
    s->c0 = vadd(s->c0, vmul(beta, vsub(s->c, s->c0)));
    s->a0 += beta * (s->a - s->a0);
    s->alpha0 = alpha;
}

enum { SF_POINTS, SF_FACEA, SF_FACEB };
typedef struct { const opoly *pA, *pB; osweep sA, sB; int type; ov2 localPoint, axis; } osepfn;

static void sep_init(osepfn *f, const ocache *cache, const opoly *pA, const osweep *sA, const opoly *pB, const osweep *sB, float t1) {
    f->pA = pA; f->pB = pB; f->sA = *sA; f->sB = *sB;
    oxf xfA = sweep_xf(&f->sA, t1), xfB = sweep_xf(&f->sB, t1);
    if (cache->count == 1) {
        f->type = SF_POINTS;
        ov2 pointA = xmul(xfA, pA->v[cache->indexA[0]]), pointB = xmul(xfB, pB->v[cache->indexB[0]]);
        f->axis = vsub(pointB, pointA);
        vnormalize(&f->axis);
        f->localPoint = V(0, 0);
    } else if (cache->indexA[0] == cache->indexA[1]) {
        f->type = SF_FACEB;
        ov2 lB1 = pB->v[cache->indexB[0]], lB2 = pB->v[cache->indexB[1]];
        f->axis = vcross_vs(vsub(lB2, lB1), 1.0f);
        vnormalize(&f->axis);
        ov2 normal = rmul(xfB.q, f->axis);
        f->localPoint = vmul(0.5f, vadd(lB1, lB2));
        ov2 pointB = xmul(xfB, f->localPoint);
        ov2 pointA = xmul(xfA, pA->v[cache->indexA[0]]);
        float s = vdot(vsub(pointA, pointB), normal);
        if (s < 0.0f) f->axis = vneg(f->axis);
    } else {
        f->type = SF_FACEA;
        ov2 lA1 = pA->v[cache->indexA[0]], lA2 = pA->v[cache->indexA[1]];
        f->axis = vcross_vs(vsub(lA2, lA1), 1.0f);
        vnormalize(&f->axis);
        ov2 normal = rmul(xfA.q, f->axis);
        f->localPoint = vmul(0.5f, vadd(lA1, lA2));
        ov2 pointA = xmul(xfA, f->localPoint);
        ov2 pointB = xmul(xfB, pB->v[cache->indexB[0]]);
        float s = vdot(vsub(pointB, pointA), normal);
        if (s < 0.0f) f->axis = vneg(f->axis);
    }
}
static float sep_find_min(const osepfn *f, int *iA, int *iB, float t) {
    oxf xfA = sweep_xf(&f->sA, t), xfB = sweep_xf(&f->sB, t);
    if (f->type == SF_POINTS) {
        ov2 axisA = rmulT(xfA.q, f->axis), axisB = rmulT(xfB.q, vneg(f->axis));
        *iA = support(f->pA, axisA); *iB = support(f->pB, axisB);
        ov2 pointA = xmul(xfA, f->pA->v[*iA]), pointB = xmul(xfB, f->pB->v[*iB]);
        return vdot(vsub(pointB, pointA), f->axis);
    } else if (f->type == SF_FACEA) {
        ov2 normal = rmul(xfA.q, f->axis);
        ov2 pointA = xmul(xfA, f->localPoint);
        ov2 axisB = rmulT(xfB.q, vneg(normal));
        *iA = -1; *iB = support(f->pB, axisB);
        ov2 pointB = xmul(xfB, f->pB->v[*iB]);
        return vdot(vsub(pointB, pointA), normal);
    } else {
        ov2 normal = rmul(xfB.q, f->axis);
        ov2 pointB = xmul(xfB, f->localPoint);
        ov2 axisA = rmulT(xfA.q, vneg(normal));
        *iB = -1; *iA = support(f->pA, axisA);
        ov2 pointA = xmul(xfA, f->pA->v[*iA]);
        return vdot(vsub(pointA, pointB), normal);
    }
}
static float sep_eval(const osepfn *f, int iA, int iB, float t) {
    oxf xfA = sweep_xf(&f->sA, t), xfB = sweep_xf(&f->sB, t);
    if (f->type == SF_POINTS) {
        ov2 pointA = xmul(xfA, f->pA->v[iA]), pointB = xmul(xfB, f->pB->v[iB]);
        return vdot(vsub(pointB, pointA), f->axis);
    } else if (f->type == SF_FACEA) {
        ov2 normal = rmul(xfA.q, f->axis);
        ov2 pointA = xmul(xfA, f->localPoint);
        ov2 pointB = xmul(xfB, f->pB->v[iB]);
        return vdot(vsub(pointB, pointA), normal);
    } else {
        ov2 normal = rmul(xfB.q, f->axis);
        ov2 pointB = xmul(xfB, f->localPoint);
        ov2 pointA = xmul(xfA, f->pA->v[iA]);
        return vdot(vsub(pointA, pointB), normal);
    }
}
enum { TOI_UNKNOWN, TOI_FAILED, TOI_OVERLAPPED, TOI_TOUCHING, TOI_SEPARATED };
static float time_of_impact(int *state, const opoly *pA, const osweep *sweepA_in, const opoly *pB, const osweep *sweepB_in, float tMax) {
    *state = TOI_UNKNOWN;
    float out_t = tMax;
    osweep sA = *sweepA_in, sB = *sweepB_in;
    sweep_normalize(&sA); sweep_normalize(&sB);
    float totalRadius = pA->radius + pB->radius;
    float target = fmax_b2(LINEAR_SLOP, totalRadius - 3.0f * LINEAR_SLOP);
    float tolerance = 0.25f * LINEAR_SLOP;
    float t1 = 0.0f;
    int iter = 0;
    ocache cache; memset(&cache, 0, sizeof(cache)); cache.count = 0;
    for (;;) {
        oxf xfA = sweep_xf(&sA, t1), xfB = sweep_xf(&sB, t1);
        float distance = gjk_distance(&cache, pA, xfA, pB, xfB);
        if (distance <= 0.0f) { *state = TOI_OVERLAPPED; out_t = 0.0f; break; }
        if (distance < target + tolerance) { *state = TOI_TOUCHING; out_t = t1; break; }
        osepfn fcn;
        sep_init(&fcn, &cache, pA, &sA, pB, &sB, t1);
        int done = 0;
        float t2 = tMax;
        int pushBackIter = 0;
        for (;;) {
            int indexA, indexB;
            float s2 = sep_find_min(&fcn, &indexA, &indexB, t2);
            if (s2 > target + tolerance) { *state = TOI_SEPARATED; out_t = tMax; done = 1; break; }
            if (s2 > target - tolerance) { t1 = t2; break; }
            float s1 = sep_eval(&fcn, indexA, indexB, t1);
            if (s1 < target - tolerance) { *state = TOI_FAILED; out_t = t1; done = 1; break; }
            if (s1 <= target + tolerance) { *state = TOI_TOUCHING; out_t = t1; done = 1; break; }
            int rootIterCount = 0;
            float a1 = t1, a2 = t2;
            for (;;) {
                float t;
                if (rootIterCount & 1) t = a1 + (target - s1) * (a2 - a1) / (s2 - s1);
                else t = 0.5f * (a1 + a2);
                ++rootIterCount;
                float s = sep_eval(&fcn, indexA, indexB, t);
                if (fabsf(s - target) < tolerance) { t2 = t; break; }
                if (s > target) { a1 = t; s1 = s; } else { a2 = t; s2 = s; }
                if (rootIterCount == 50) break;
            }
            ++pushBackIter;
            if (pushBackIter == MAX_POLY_VERTS) break;
        }
        ++iter;
        if (done) break;
        if (iter == 20) { *state = TOI_FAILED; out_t = t1; break; }
    }
    return out_t;
}

/* b2Island::SolveTOI for the car + touching walls at the TOI pose */
static void island_solve_toi(oworld *w, const owalls *W, const olistener *L, const int *cidx, int n, float subdt, int velIters) {
    obodystate A; A.c = w->c; A.a = w->a; A.v = w->v; A.w = w->w;
    ovc vc[MAX_TOI_CONTACTS];
    cs_init(vc, n, w, cidx, W, 0, 1.0f);
    for (int it = 0; it < 20; ++it) { if (cs_solve_position(vc, n, &A, 1)) break; }
    w->c0 = A.c; w->a0 = A.a;
    cs_init_velocity(vc, n, w, &A);
    for (int it = 0; it < velIters; ++it) cs_solve_velocity(vc, n, &A);
    integrate_positions(&A, subdt);
    w->c = A.c; w->a = A.a; w->v = A.v; w->w = A.w;
    sync_transform(w);
    report(vc, n, L);
}

/* b2World::SolveTOI */
static void solve_toi(oworld *w, const owalls *W, const olistener *L, float dt, int velIters) {
    opoly pa; car_poly(&pa);
    w->alpha0 = 0.0f;
    for (int i = 0; i < w->nct; ++i) { w->ct[i].flags &= ~(OC_TOI | OC_ISLAND); w->ct[i].toiCount = 0; w->ct[i].toi = 1.0f; }
    for (;;) {
        int minC = -1; float minAlpha = 1.0f;
        for (int i = 0; i < w->nct; ++i) {
            ocontact *c = &w->ct[i];
            if (!(c->flags & OC_ENABLED)) continue;
            if (c->toiCount > MAX_SUBSTEPS) continue;
            float alpha = 1.0f;
            if (c->flags & OC_TOI) alpha = c->toi;
            else {
                if (!w->awake) continue;
                float alpha0 = w->alpha0;
                opoly pb; wall_poly(&pb, W, c->wall);
                osweep sA = { w->c0, w->c, w->a0, w->a, w->alpha0 };
                osweep sB = { W->p[c->wall], W->p[c->wall], W->angle[c->wall], W->angle[c->wall], 0.0f };
                int state;
                float beta = time_of_impact(&state, &pa, &sA, &pb, &sB, 1.0f);
                if (state == TOI_TOUCHING) alpha = fmin_b2(alpha0 + (1.0f - alpha0) * beta, 1.0f);
                else alpha = 1.0f;
                c->toi = alpha; c->flags |= OC_TOI;
            }
            if (alpha < minAlpha) { minC = i; minAlpha = alpha; }
        }
        if (minC < 0 || 1.0f - 10.0f * FLT_EPSILON < minAlpha) break;
        /* advance the car (walls are static: b2Body::Advance is a no-op on them) */
        ov2 bc0 = w->c0, bc = w->c; float ba0 = w->a0, ba = w->a, balpha0 = w->alpha0;
        {
            osweep s = { w->c0, w->c, w->a0, w->a, w->alpha0 };
            sweep_advance(&s, minAlpha);
            w->c0 = s.c0; w->a0 = s.a0; w->alpha0 = s.alpha0;
            w->c = w->c0; w->a = w->a0;
            sync_transform(w);
        }
        int minWall = w->ct[minC].wall;
        contact_update(w, minC, W, L);
        /* contact_update never reorders the list, minC stays valid */
        w->ct[minC].flags &= ~OC_TOI;
        ++w->ct[minC].toiCount;
        if (!(w->ct[minC].flags & OC_ENABLED) || !(w->ct[minC].flags & OC_TOUCH)) {
            w->ct[minC].flags &= ~OC_ENABLED;
            w->c0 = bc0; w->c = bc; w->a0 = ba0; w->a = ba; w->alpha0 = balpha0;
            sync_transform(w);
            continue;
        }
        set_awake(w);
        int cidx[MAX_TOI_CONTACTS], n = 0;
        cidx[n++] = minC; w->ct[minC].flags |= OC_ISLAND;
        (void)minWall;
        for (int i = 0; i < w->nct; ++i) {
            if (n == MAX_TOI_CONTACTS) break;
            ocontact *c = &w->ct[i];
            if (c->flags & OC_ISLAND) continue;
            contact_update(w, i, W, L);
            if (!(c->flags & OC_ENABLED)) continue;
            if (!(c->flags & OC_TOUCH)) continue;
            c->flags |= OC_ISLAND;
            cidx[n++] = i;
        }
        float subdt = (1.0f - minAlpha) * dt;
        island_solve_toi(w, W, L, cidx, n, subdt, velIters);
        sync_fixtures(w);
        for (int i = 0; i < w->nct; ++i) w->ct[i].flags &= ~(OC_TOI | OC_ISLAND);
        find_new_contacts(w, W);
    }
}

void ob_step(oworld *w, const owalls *W, const olistener *L, float dt, int velIters, int posIters) {
    float inv_dt = dt > 0.0f ? 1.0f / dt : 0.0f;
    float dtRatio = w->inv_dt0 * dt;
    collide(w, W, L);
    solve(w, W, L, dt, dtRatio, velIters, posIters);
    solve_toi(w, W, L, dt, velIters);
    w->inv_dt0 = inv_dt;
    w->force = V(0.0f, 0.0f); w->torque = 0.0f;
}

void ob_world_init(oworld *w, const owalls *W, ov2 pos, float angle) {
    memset(w, 0, sizeof(*w));
    ob_rot_set(&w->xf.q, angle);
    w->xf.p = pos;
    w->c = xmul(w->xf, V(0.0f, 0.0f)); w->a = angle; w->c0 = w->c; w->a0 = angle;
    w->awake = 1;
    opoly cp; car_poly(&cp);
    oaabb a = poly_aabb(&cp, w->xf);
    ov2 r = V(AABB_EXT, AABB_EXT);
    w->fat.lo = vsub(a.lo, r); w->fat.hi = vadd(a.hi, r);
    w->moved = 1;
    find_new_contacts(w, W);    /* the first Step's e_newFixture FindNewContacts */
}

/* b2Body::SetTransform (pybox2d body.position / body.angle setters) */
void ob_set_transform(oworld *w, const owalls *W, ov2 pos, float angle) {
    ob_rot_set(&w->xf.q, angle);
    w->xf.p = pos;
    w->c = xmul(w->xf, V(0.0f, 0.0f)); w->a = angle;
    w->c0 = w->c; w->a0 = angle;
    move_proxy(w, w->xf, w->xf);
    find_new_contacts(w, W);
}

/* b2PolygonShape::RayCast per wall, b2World::RayCast clipping semantics (min fraction) */
float ob_raycast(const owalls *W, ov2 p1w, ov2 p2w) {
    float best = -1.0f;
    for (int j = 0; j < W->n; ++j) {
        oxf xf = wall_xf(W, j);
        opoly p; wall_poly(&p, W, j);
        ov2 p1 = rmulT(xf.q, vsub(p1w, xf.p));
        ov2 p2 = rmulT(xf.q, vsub(p2w, xf.p));
        ov2 d = vsub(p2, p1);
        float lower = 0.0f, upper = 1.0f;
        int index = -1, ok = 1;
        for (int i = 0; i < p.count; ++i) {
            float numerator = vdot(p.n[i], vsub(p.v[i], p1));
            float denominator = vdot(p.n[i], d);
            if (denominator == 0.0f) {
                if (numerator < 0.0f) { ok = 0; break; }
            } else {
                if (denominator < 0.0f && numerator < lower * denominator) { lower = numerator / denominator; index = i; }
                else if (denominator > 0.0f && numerator < upper * denominator) { upper = numerator / denominator; }
            }
            if (upper < lower) { ok = 0; break; }
        }
        if (!ok || index < 0) continue;
        if (best < 0.0f || lower < best) best = lower;
    }
    return best;
}

/* CarPhysics._check_wall_collision AABB query (src/car_physics.py:470-524) */
int ob_query_on_wall(const owalls *W, double px, double py, double radius) {
    oaabb q; q.lo = V((float)(px - radius), (float)(py - radius)); q.hi = V((float)(px + radius), (float)(py + radius));
    ov2 center = V((float)px, (float)py);
    for (int j = 0; j < W->n; ++j) {
        if (!overlap(W->fat[j], q)) continue;
        oxf xf = wall_xf(W, j);
        opoly p; wall_poly(&p, W, j);
        ov2 pl = rmulT(xf.q, vsub(center, xf.p));
        int inside = 1;
        for (int i = 0; i < p.count; ++i) { if (vdot(p.n[i], vsub(pl, p.v[i])) > 0.0f) { inside = 0; break; } }
        if (inside) return 1;
        for (int i = 0; i < p.count; ++i) {
            ov2 v = xmul(xf, p.v[i]);
            double dx = px - (double)v.x, dy = py - (double)v.y;
            double dist = pow(dx * dx + dy * dy, 0.5);
            if (dist < radius) return 1;
        }
    }
    return 0;
}
