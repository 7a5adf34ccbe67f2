/*
 * oracle/nascar_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's CarEnv hot path (heihachi78/NascarGymnasium
 * @ /root/reference).  It is the parity CHECKER for the HIP product path and the
 * `cpu_baseline` leg of bench.py; nothing in nascargymnasium_amd/ links or calls
 * it.  Float64 where the reference computes in Python floats, float32 where the
 * reference goes through Box2D (b2_oracle.c) or numpy float32.
 *
 * Pinned against golden vectors generated from the reference's own Python
 * (tests/golden/, oracle/gen_golden.py): track tables + wall builder, the
 * vehicle/tyre model, the lap timer and the env reward/disable/termination
 * logic.  The Box2D internals (b2_oracle.c) are parity-unpinned.
 *
 * Each function cites the reference file:line it restates.
 */
#include "b2_oracle.h"
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>

#define EXPORT __attribute__((visibility("default")))

/* ---------------- constants: src/constants (same double expressions) ---- */
#define PI_ M_PI
static const double CAR_MASS = 1500.0;
static const double GRAVITY_MS2 = 9.81;
static const double CAR_WHEELBASE = 2.794;
static const double CAR_MAX_TORQUE = 820.0;
#define CAR_MAX_POWER (670.0 * 745.7)
#define CAR_MAX_SPEED_MS (200.0 * 0.44704)
#define DRAG_CONSTANT (0.5 * 1.225 * 0.38 * 2.5)
#define ROLLING_RESISTANCE_FORCE (0.015 * CAR_MASS * GRAVITY_MS2)
#define MAX_TYRE_LOAD (CAR_MASS * GRAVITY_MS2 * 2.0)
#define STATIC_LOAD_PER_TYRE (CAR_MASS * GRAVITY_MS2 / 4.0)
#define RAD_PER_DEG (PI_ / 180.0)       /* CPython math.radians: x * (pi/180) */
#define DEG_PER_RAD (180.0 / PI_)       /* CPython math.degrees: x * (180/pi) */
#define PHYS_DT (1.0 / 60.0)

EXPORT double or_dbg[32];
EXPORT int or_dbg_car = -1;
static _Thread_local int g_cur_car = -2;   // debug tap selector (thread-local: bench runs oracle shards on threads)
#define ODBG(slot, val) do { if (g_cur_car == or_dbg_car) or_dbg[slot] = (double)(val); } while (0)
static inline double pymin(double a, double b) { return b < a ? b : a; }
static inline double pymax(double a, double b) { return b > a ? b : a; }
static inline double npclip(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
/* Python `x ** 2` is glibc pow(x, 2.0) (CPython float_pow), which is not always x*x */
static inline double P2(double x) { return pow(x, 2.0); }

/* ---------------- track: src/track_generator.py --------------------------- */
enum { SEG_GRID, SEG_STARTLINE, SEG_STRAIGHT, SEG_FINISHLINE, SEG_CURVE };
typedef struct {
    int type; double length, sx, sy, ex, ey, width, curve_angle, curve_radius; int dir_left;
    double start_heading, end_heading, banking;
} oseg;

typedef struct {
    int nseg; oseg seg[64];
    double width, total_length, cur_x, cur_y, cur_heading;
    /* wall table (src/car_physics.py:118-339) */
    owalls W;
    double *wall_cx, *wall_cy, *wall_ang, *wall_hl;  /* double values before the float cast */
    int startline;       /* index of the first STARTLINE segment or -1 */
    int has_banking;
    double start_x, start_y;
} otrack;

/* Track.add_segment (src/track_generator.py:66-115) */
static void add_segment(otrack *t, int type, double length, double curve_angle, double curve_radius, int left, double banking) {
    oseg s; memset(&s, 0, sizeof(s));
    double sx = t->cur_x, sy = t->cur_y, sh = t->cur_heading, ex, ey, eh;
    if (curve_angle == 0.0) {
        eh = sh;
        double hr = sh * RAD_PER_DEG;
        ex = sx + length * cos(hr); ey = sy + length * sin(hr);
    } else {
        type = SEG_CURVE;
        double shr = sh * RAD_PER_DEG, car = curve_angle * RAD_PER_DEG;
        double turn = left ? 1.0 : -1.0;
        double perp = shr + turn * PI_ / 2;
        double cx = sx + curve_radius * cos(perp), cy = sy + curve_radius * sin(perp);
        eh = sh + turn * curve_angle;
        double a0 = shr - turn * PI_ / 2;
        double a1 = a0 + turn * car;
        ex = cx + curve_radius * cos(a1); ey = cy + curve_radius * sin(a1);
        length = fabs(curve_radius * (curve_angle * RAD_PER_DEG));
    }
    s.type = type; s.length = length; s.sx = sx; s.sy = sy; s.ex = ex; s.ey = ey; s.width = t->width;
    s.curve_angle = curve_angle; s.curve_radius = curve_radius; s.dir_left = left;
    s.start_heading = sh; s.end_heading = eh; s.banking = banking;
    t->seg[t->nseg++] = s;
    t->total_length += length;
    t->cur_x = ex; t->cur_y = ey; t->cur_heading = eh;
}

/* TrackLoader.load_track (src/track_generator.py:305-405); returns 0 on success */
static int load_track(otrack *t, const char *path, char *err, size_t errlen) {
    FILE *f = fopen(path, "r");
    if (!f) { snprintf(err, errlen, "Track file not found: %s", path); return -1; }
    memset(t, 0, sizeof(*t));
    t->width = 20.0;
    char line[512];
    while (fgets(line, sizeof line, f)) {
        for (char *p = line; *p; ++p) *p = (char)toupper((unsigned char)*p);
        char *hash = strchr(line, '#');
        if (hash) *hash = 0;
        char *tok[8]; int nt = 0;
        for (char *p = strtok(line, " \t\r\n\v\f"); p && nt < 8; p = strtok(NULL, " \t\r\n\v\f")) tok[nt++] = p;
        if (nt == 0) continue;
        if (t->nseg >= 63) { fclose(f); snprintf(err, errlen, "too many segments"); return -1; }
        if (!strcmp(tok[0], "WIDTH")) {
            if (nt != 2) { fclose(f); snprintf(err, errlen, "WIDTH command requires exactly one argument"); return -1; }
            t->width = strtod(tok[1], NULL);
        } else if (!strcmp(tok[0], "GRID")) add_segment(t, SEG_GRID, 100.0, 0, 0, 0, 0.0);
        else if (!strcmp(tok[0], "STARTLINE")) add_segment(t, SEG_STARTLINE, 5.0, 0, 0, 0, 0.0);
        else if (!strcmp(tok[0], "FINISHLINE")) add_segment(t, SEG_FINISHLINE, 5.0, 0, 0, 0, 0.0);
        else if (!strcmp(tok[0], "STRAIGHT")) {
            if (nt < 2 || nt > 3) { fclose(f); snprintf(err, errlen, "STRAIGHT command requires 1-2 arguments"); return -1; }
            double len = strtod(tok[1], NULL), bank = nt == 3 ? strtod(tok[2], NULL) : 0.0;
            if (bank < -45 || bank > 45) { fclose(f); snprintf(err, errlen, "Banking angle must be between -45 and 45 degrees"); return -1; }
            add_segment(t, SEG_STRAIGHT, len, 0, 0, 0, bank);
        } else if (!strcmp(tok[0], "LEFT") || !strcmp(tok[0], "RIGHT")) {
            if (nt < 3 || nt > 4) { fclose(f); snprintf(err, errlen, "curve command requires 2-3 arguments"); return -1; }
            double ang = strtod(tok[1], NULL), rad = strtod(tok[2], NULL), bank = nt == 4 ? strtod(tok[3], NULL) : 0.0;
            if (ang <= 0 || ang > 360) { fclose(f); snprintf(err, errlen, "Curve angle must be between 0 and 360 degrees"); return -1; }
            if (rad <= 0) { fclose(f); snprintf(err, errlen, "Curve radius must be positive"); return -1; }
            if (bank < -45 || bank > 45) { fclose(f); snprintf(err, errlen, "Banking angle must be between -45 and 45 degrees"); return -1; }
            add_segment(t, SEG_CURVE, 0, ang, rad, tok[0][0] == 'L', bank);
        } else { fclose(f); snprintf(err, errlen, "Unknown command: %s", tok[0]); return -1; }
    }
    fclose(f);
    return 0;
}

/* ---- wall builder: CarPhysics._create_track_walls (src/car_physics.py:118-339) ---- */
typedef struct { int n, cap; double *cx, *cy, *ang, *hl; } wlist;
static void wl_push(wlist *l, double cx, double cy, double ang, double hl) {
    if (l->n == l->cap) {
        l->cap = l->cap ? l->cap * 2 : 1024;
        l->cx = realloc(l->cx, sizeof(double) * l->cap); l->cy = realloc(l->cy, sizeof(double) * l->cap);
        l->ang = realloc(l->ang, sizeof(double) * l->cap); l->hl = realloc(l->hl, sizeof(double) * l->cap);
    }
    l->cx[l->n] = cx; l->cy[l->n] = cy; l->ang[l->n] = ang; l->hl[l->n] = hl; l->n++;
}
/* _create_wall_body_from_line (src/car_physics.py:280-339) */
static void wall_from_line(wlist *l, double x1, double y1, double x2, double y2) {
    double cx = (x1 + x2) / 2, cy = (y1 + y2) / 2;
    double length = pow(P2(x2 - x1) + P2(y2 - y1), 0.5);
    if (length < 0.1) return;
    double angle = atan2(y2 - y1, x2 - x1);
    wl_push(l, cx, cy, angle, length / 2);
}
static void build_walls(otrack *t) {
    wlist l; memset(&l, 0, sizeof(l));
    for (int k = 0; k < t->nseg; ++k) {
        const oseg *s = &t->seg[k];
        if (s->type == SEG_CURVE) {
            /* _create_curved_walls / _generate_curve_wall_points (:185-278) */
            if (s->curve_radius <= 0 || s->curve_angle <= 0) continue;
            double hw = s->width / 2, shr = s->start_heading * RAD_PER_DEG, car = s->curve_angle * RAD_PER_DEG;
            double turn = s->dir_left ? 1.0 : -1.0;
            double perp = shr + turn * PI_ / 2;
            double cx = s->sx + s->curve_radius * cos(perp), cy = s->sy + s->curve_radius * sin(perp);
            double ri = s->dir_left ? s->curve_radius - hw : s->curve_radius + hw;
            double ro = s->dir_left ? s->curve_radius + hw : s->curve_radius - hw;
            double a0 = shr - turn * PI_ / 2;
            int nsd = (int)(fabs(s->curve_angle) / 1.0);
            int ns = nsd < 180 ? nsd : 180; if (ns < 8) ns = 8;
            double *ix = malloc(sizeof(double) * (ns + 1)), *iy = malloc(sizeof(double) * (ns + 1));
            double *ox = malloc(sizeof(double) * (ns + 1)), *oy = malloc(sizeof(double) * (ns + 1));
            int ni = 0, no = 0;
            for (int i = 0; i <= ns; ++i) {
                double tt = (double)i / ns;
                double angle = a0 + turn * car * tt;
                if (ri > 0) { ix[ni] = cx + ri * cos(angle); iy[ni] = cy + ri * sin(angle); ni++; }
                ox[no] = cx + ro * cos(angle); oy[no] = cy + ro * sin(angle); no++;
            }
            if (ni >= 2 && no >= 2) {
                for (int i = 0; i < ni - 1; ++i) wall_from_line(&l, ix[i], iy[i], ix[i + 1], iy[i + 1]);
                for (int i = 0; i < no - 1; ++i) wall_from_line(&l, ox[i], oy[i], ox[i + 1], oy[i + 1]);
            }
            free(ix); free(iy); free(ox); free(oy);
        } else {
            /* _create_straight_walls (:137-183) */
            double hw = s->width / 2;
            double sl = sqrt(P2(s->ex - s->sx) + P2(s->ey - s->sy));
            double pdx, pdy;
            if (sl > 0) { double dx = (s->ex - s->sx) / sl, dy = (s->ey - s->sy) / sl; pdx = -dy; pdy = dx; }
            else { pdx = 0; pdy = 1; }
            wall_from_line(&l, s->sx + pdx * hw, s->sy + pdy * hw, s->ex + pdx * hw, s->ey + pdy * hw);
            wall_from_line(&l, s->sx - pdx * hw, s->sy - pdy * hw, s->ex - pdx * hw, s->ey - pdy * hw);
        }
    }
    owalls *W = &t->W;
    W->n = l.n;
    W->p = calloc((size_t)l.n, sizeof(ov2)); W->angle = calloc((size_t)l.n, sizeof(float)); W->q = calloc((size_t)l.n, sizeof(orot));
    W->hx = calloc((size_t)l.n, sizeof(float)); W->hy = calloc((size_t)l.n, sizeof(float));
    W->fat = calloc((size_t)l.n, sizeof(oaabb)); W->key = calloc((size_t)l.n, sizeof(int));
    char (*keys)[64] = calloc((size_t)l.n, 64);
    int nkeys = 0;
    for (int j = 0; j < l.n; ++j) {
        W->p[j].x = (float)l.cx[j]; W->p[j].y = (float)l.cy[j];
        W->angle[j] = (float)l.ang[j];
        ob_rot_set(&W->q[j], W->angle[j]);
        W->hx[j] = (float)l.hl[j]; W->hy[j] = (float)(1.0 / 2);
        /* b2PolygonShape::ComputeAABB + b2DynamicTree::CreateProxy fattening */
        float hx = W->hx[j], hy = W->hy[j];
        ov2 vs[4] = { {-hx, -hy}, {hx, -hy}, {hx, hy}, {-hx, hy} };
        float lx = 0, ly = 0, ux = 0, uy = 0;
        for (int i = 0; i < 4; ++i) {
            float x = (W->q[j].c * vs[i].x - W->q[j].s * vs[i].y) + W->p[j].x;
            float y = (W->q[j].s * vs[i].x + W->q[j].c * vs[i].y) + W->p[j].y;
            if (i == 0) { lx = ux = x; ly = uy = y; }
            else { lx = x < lx ? x : lx; ly = y < ly ? y : ly; ux = ux > x ? ux : x; uy = uy > y ? uy : y; }
        }
        const float r = 2.0f * 0.005f;
        W->fat[j].lo.x = (lx - r) - 0.1f; W->fat[j].lo.y = (ly - r) - 0.1f;
        W->fat[j].hi.x = (ux + r) + 0.1f; W->fat[j].hi.y = (uy + r) + 0.1f;
        /* listener key f"wall_{pos.x:.1f}_{pos.y:.1f}" (src/car_physics.py:747) */
        char k[64]; snprintf(k, sizeof k, "wall_%.1f_%.1f", (double)W->p[j].x, (double)W->p[j].y);
        int id = -1;
        for (int q = 0; q < nkeys; ++q) if (!strcmp(keys[q], k)) { id = q; break; }
        if (id < 0) { strcpy(keys[nkeys], k); id = nkeys++; }
        W->key[j] = id;
    }
    free(keys);
    t->wall_cx = l.cx; t->wall_cy = l.cy; t->wall_ang = l.ang; t->wall_hl = l.hl;
    t->startline = -1;
    for (int k = 0; k < t->nseg; ++k) if (t->seg[k].type == SEG_STARTLINE) { t->startline = k; break; }
    t->has_banking = 0;
    for (int k = 0; k < t->nseg; ++k) if (fabs(t->seg[k].banking) >= 0.1) { t->has_banking = 1; break; }
    /* CarEnv._load_track start position: first GRID/STARTLINE segment start (src/car_env.py:235-241) */
    t->start_x = 0; t->start_y = 0;
    for (int k = 0; k < t->nseg; ++k) if (t->seg[k].type == SEG_GRID || t->seg[k].type == SEG_STARTLINE) { t->start_x = t->seg[k].sx; t->start_y = t->seg[k].sy; break; }
}

/* ---------------- per-car state ------------------------------------------- */
typedef struct {
    oworld w;
    /* Car (src/car.py:140-189) */
    double thr_in, brk_in, str_in, thr, brk, steer;
    double rpm, pvx, pvy;
    double acc[10][2]; int acc_len, acc_head;
    double lfm, slip, bank;
    /* TyreManager / Tyre (src/tyre_manager.py, src/tyre.py), order FL FR RL RR */
    double load[4], temp[4], wear[4], fric[4];
    /* CarCollisionListener (src/car_physics.py:693-864) */
    int imp_present; double imp;
    int nact; int act_key[OB_MAXC]; float act_nx[OB_MAXC], act_ny[OB_MAXC];
    const owalls *W;
    /* LapTimer (src/lap_timer.py:36-59) */
    int lt_timing; double lt_start, lt_cur; int lt_has_last, lt_has_best; double lt_last, lt_best;
    int lt_crossed, lt_has_pos; double lt_px, lt_py; int lt_laps; double lt_dist;
    /* CarEnv bookkeeping (src/car_env.py) */
    int disabled, just_disabled;
    double cum_impact, stuck_dur; int has_stuck_start; double stuck_sx, stuck_sy;
    double prev_px, prev_py;
    double prog_hist, back, prev_back; int first_step; int prev_laps;
    float cum_reward, cum_reward_info;
    /* last step outputs */
    float obs[38]; float reward; double imp_at_obs;
} ocar;

typedef struct {
    otrack trk;
    int E, C, reset_on_lap;
    double start_x, start_y, start_angle;
    ocar *car;                 /* E*C */
    double *sim_time; int *created, *pending, *term_reason, *terminated, *truncated;
    char err[256];
} oenv;

/* ---------------- listener -------------------------------------------------- */
static void lis_begin(void *u, int wall, ov2 n) {
    ocar *c = (ocar *)u; int key = c->W->key[wall];
    int found = -1;
    for (int i = 0; i < c->nact; ++i) if (c->act_key[i] == key) { found = i; break; }
    if (found >= 0) { c->act_nx[found] = n.x; c->act_ny[found] = n.y; }
    else if (c->nact < OB_MAXC) { c->act_key[c->nact] = key; c->act_nx[c->nact] = n.x; c->act_ny[c->nact] = n.y; c->nact++; }
    if (!c->imp_present) { c->imp_present = 1; c->imp = 0.0; }
}
static void lis_end(void *u, int wall) {
    ocar *c = (ocar *)u; int key = c->W->key[wall];
    for (int i = 0; i < c->nact; ++i) if (c->act_key[i] == key) {
        memmove(&c->act_key[i], &c->act_key[i + 1], sizeof(int) * (size_t)(c->nact - i - 1));
        memmove(&c->act_nx[i], &c->act_nx[i + 1], sizeof(float) * (size_t)(c->nact - i - 1));
        memmove(&c->act_ny[i], &c->act_ny[i + 1], sizeof(float) * (size_t)(c->nact - i - 1));
        c->nact--; break;
    }
    if (c->nact == 0) { c->imp_present = 1; c->imp = 0.0; }
}
static void lis_post(void *u, int count, const float *ni) {
    ocar *c = (ocar *)u;
    if (count <= 0) return;
    double total = 0.0;
    for (int i = 0; i < count; ++i) total += (double)ni[i];
    if (c->imp_present) c->imp = pymax(c->imp, total);
}

/* ---------------- tyres ----------------------------------------------------- */
/* Tyre.get_grip_coefficient (src/tyre.py:197-224) */
static double tyre_grip(double T, double wear) {
    double tg;
    if (85.0 <= T && T <= 105.0) tg = 1.5;
    else {
        double dev = T < 85.0 ? 85.0 - T : T - 105.0;
        double g = 1.5 - dev * 0.02;
        tg = pymax(0.8, g);
    }
    double wf = 1.0 - (wear / 100.0) * (1.0 - 0.5);
    return tg * wf;
}
/* TyreManager.get_total_grip_coefficient (src/tyre_manager.py:211-222) */
static double total_grip(const ocar *c) {
    double tg = 0.0, tw = 0.0;
    for (int i = 0; i < 4; ++i) { tg += tyre_grip(c->temp[i], c->wear[i]) * c->load[i]; tw += c->load[i]; }
    return tw > 0 ? tg / tw : 0.0;
}
/* Tyre._update_temperature / _update_wear (src/tyre.py:85-172) */
static void tyre_update(ocar *c, int i, double dt, double load, double ff, double speed, double lat, double slip) {
    c->load[i] = load;
    double ns = pymin(speed / CAR_MAX_SPEED_MS, 2.0);
    double sf = 1.0 + P2(ns);
    double fp = fabs(ff) * 0.040 * sf;
    double ah = 0.0;
    if (speed > 50.0) ah = P2(speed) * 0.0002;
    double th = (fp + ah) * dt / 125.0;
    double td = c->temp[i] - 25.0;
    double ce = 0.01;
    if (speed > 50.0) { double cr = pymin(0.8, speed / 100.0); ce *= (1.0 - cr * 0.5); }
    double cool = td * ce;
    double tdec = cool * dt;
    c->temp[i] += th - tdec;
    c->temp[i] = pymax(25.0, pymin(120.0, c->temp[i]));
    double T = c->temp[i];
    double fwr = fabs(ff) * 0.00001;
    double tm;
    if (85.0 <= T && T <= 105.0) tm = 1.0;
    else if (T > 105.0) tm = 1.0 + ((T - 105.0) / 20.0);
    else tm = 1.0 + ((85.0 - T) / 30.0);
    double lf = load / STATIC_LOAD_PER_TYRE;
    double lm = pymax(0.5, lf);
    double wf = pymax(1.0, T / 80.0);
    double skmh = speed * 3.6;
    double swf = 1.0 + (skmh / 400.0) * 3.0;
    swf = pymin(swf, 3.0);
    double lat_g = fabs(lat) / 9.81;
    double cwf;
    if (lat_g > 2.0) { double ex = lat_g - 2.0; cwf = 1.0 + (ex * 1.5); cwf = pymin(cwf, 2.5); }
    else cwf = 1.0;
    double slwf = 1.0 + (fabs(slip) / 45.0) * (3.0 - 1.0);
    slwf = pymin(slwf, 3.0);
    double tot = tm * lm * wf * swf * cwf * slwf;
    double rate = fwr * tot;
    c->wear[i] += rate * dt;
    c->wear[i] = pymin(100.0, c->wear[i]);
}
/* TyreManager._calculate_weight_transfer (src/tyre_manager.py:99-202) */
static void weight_transfer(ocar *c, double lon, double lat, double speed, double out[4]) {
    double sw = CAR_MASS * GRAVITY_MS2, sfl = sw * 0.5, srl = sw * 0.5;
    double aero = 0.0;
    if (speed > 50.0) {
        double sf = P2(speed / 50.0);
        double calc = 0.12 * sf * CAR_MASS * GRAVITY_MS2;
        double mx = 1.5 * CAR_MASS * GRAVITY_MS2;
        aero = pymin(calc, mx);
    }
    double ar = aero * 0.6, af = aero * (1.0 - 0.6);
    double bf = sfl + af, br = srl + ar, te = sw + aero;
    double rl = lon * te * 0.02;
    double mf = bf * 0.95, mb = br * 0.95;
    double lt = rl > 0 ? pymin(rl, mf) : pymax(rl, -mb);
    double ft = bf - lt, rt = br + lt;
    double rlat = lat * te * 0.01;
    double mltf = (ft / 2.0) - 200.0, mltr = (rt / 2.0) - 200.0;
    double mlt = pymin(mltf, mltr);
    double latt = mlt > 0 ? pymax(-mlt, pymin(mlt, rlat)) : 0.0;
    double raw[4] = { ft / 2.0 - latt / 2.0, ft / 2.0 + latt / 2.0, rt / 2.0 - latt / 2.0, rt / 2.0 + latt / 2.0 };
    double con[4], deficit = 0.0, excess = 0.0;
    for (int i = 0; i < 4; ++i) {
        if (raw[i] < 50.0) { con[i] = 50.0; deficit += 50.0 - raw[i]; }
        else { con[i] = raw[i]; excess += raw[i] - 50.0; }
    }
    if (deficit > 0.0 && excess > 0.0) {
        double fct = deficit / excess;
        for (int i = 0; i < 4; ++i) {
            if (raw[i] >= 50.0) { double e = con[i] - 50.0; out[i] = pymax(50.0, con[i] - e * fct); }
            else out[i] = con[i];
        }
    } else for (int i = 0; i < 4; ++i) out[i] = con[i];
    (void)c;
}

/* Car._add_lateral_force_heating (src/car.py:761-827) */
static void lateral_heating(ocar *c, double ff[4], double speed) {
    if (speed < 2.0) return;
    double shm = 1.0;
    if (c->slip > 5.0) { double ex = c->slip - 5.0; shm = 2.2 + (0.04 * P2(ex)); shm = pymin(shm, 8.0); }
    double base = c->lfm * 0.05 * shm;
    double flh = base * 0.5 / 2.0, rlh = base * 0.5 / 2.0;
    if (fabs(c->steer) > 0.01 && speed > 3.0) {
        int of, orr, inf, inr;
        if (c->steer < 0) { of = 0; orr = 2; inf = 1; inr = 3; }
        else { of = 1; orr = 3; inf = 0; inr = 2; }
        double ofb = c->load[of] * 0.001, orb = c->load[orr] * 0.001;
        ff[of] += flh * 1.5 + ofb;
        ff[orr] += rlh * 1.5 + orb;
        ff[inf] += flh * 0.5;
        ff[inr] += rlh * 0.5;
    } else { ff[0] += flh; ff[1] += flh; ff[2] += rlh; ff[3] += rlh; }
}
/* Car._update_friction_forces (src/car.py:702-759) */
static void update_friction(ocar *c, double df) {
    double speed = (double)sqrtf(c->w.v.x * c->w.v.x + c->w.v.y * c->w.v.y);
    double rear, front;
    if (c->thr > 0.01 && speed > 50.0) { double fa = pymin(0.3, speed / 200.0); rear = df * (1.0 - fa); front = df * fa / 2.0; }
    else { rear = c->thr > 0.01 ? df : 0.0; front = 0.0; }
    double bf = 0.0;
    if (c->brk > 0.01) {
        double mbf = CAR_MASS * 14.0 * c->brk, base = mbf / 4.0;
        if (speed <= 1.0) { double sf = 0.05 + (1.0 - 0.05) * (speed / 1.0); bf = base * sf; }
        else bf = base;
    }
    double rf = 0.0;
    if (speed > 0.1) rf = ROLLING_RESISTANCE_FORCE / 4.0;
    double ff[4] = { front + bf + rf, front + bf + rf, rear / 2.0 + bf + rf, rear / 2.0 + bf + rf };
    lateral_heating(c, ff, speed);
    memcpy(c->fric, ff, sizeof ff);
}

static inline double f32len(ov2 v) { return (double)sqrtf(v.x * v.x + v.y * v.y); }
static inline ov2 OV(double x, double y) { ov2 r; r.x = (float)x; r.y = (float)y; return r; }

/* Car.update_physics (src/car.py:329-387) with the force helpers (:389-700) */
static void car_update_physics(ocar *c, double dt) {
    oworld *w = &c->w;
    c->thr = c->thr_in; c->brk = c->brk_in; c->steer = c->str_in * (45.0 * RAD_PER_DEG);
    /* _update_engine_rpm (:311-327) */
    {
        double target = 1000.0 + (800.0 * c->thr_in);
        double diff = target - c->rpm;
        c->rpm += diff * pymin(1.0, dt * 3000.0 / fabs(diff + 0.1));
        c->rpm = pymax(600.0, pymin(9500.0, c->rpm));
    }
    /* _apply_engine_force (:389-449) */
    {
        double speed = f32len(w->v);
        double rpm = c->rpm < 1000.0 ? 1000.0 : (c->rpm > 9000.0 ? 9000.0 : c->rpm);
        double tf = rpm <= 5500.0 ? 0.7 + 0.3 * (rpm - 1000.0) / (5500.0 - 1000.0)
                                  : 1.0 - 0.6 * (rpm - 5500.0) / (9000.0 - 5500.0);
        double torque = CAR_MAX_TORQUE * tf * c->thr;
        double wheel = torque * 7.5;
        double tlf = wheel / 0.35;
        double ef;
        if (speed > 12.0) {
            double plf = (CAR_MAX_POWER * c->thr) / speed;
            if (speed <= 25.0) {
                double nsd = (speed - 12.0) / (25.0 - 12.0);
                double ex = 1.0 - exp(-2.0 * nsd);
                double blend = pymax(0.05, pymin(0.75, ex));
                ef = tlf * (1.0 - blend) + plf * blend;
            } else ef = tlf * (1.0 - 0.75) + plf * 0.75;
        } else ef = tlf;
        double grip = total_grip(c);
        double sfac = 1.0 - pymin(0.4, fabs(c->steer) * 1.5);
        double mx = CAR_MASS * GRAVITY_MS2 * grip * sfac;
        ef = pymin(ef, mx);
        /* GetWorldVector((1,0)) = b2Mul(q, (1,0)) in float32 */
        double fx = (double)(w->xf.q.c * 1.0f - w->xf.q.s * 0.0f), fy = (double)(w->xf.q.s * 1.0f + w->xf.q.c * 0.0f);
        double Fx = ef * fx, Fy = ef * fy;
        double rff = pymin(2000.0, fabs(ef) / 2.0);
        update_friction(c, rff);
        ODBG(0, ef); ODBG(1, Fx); ODBG(2, Fy); ODBG(3, speed); ODBG(4, c->rpm); ODBG(5, total_grip(c));

        /* GetWorldPoint((-wheelbase/2, 0)) in float32 */
        float lx = (float)(-CAR_WHEELBASE / 2), ly = 0.0f;
        ov2 pt; pt.x = (w->xf.q.c * lx - w->xf.q.s * ly) + w->xf.p.x; pt.y = (w->xf.q.s * lx + w->xf.q.c * ly) + w->xf.p.y;
        ob_apply_force(w, OV(Fx, Fy), pt);
    }
    /* _apply_brake_force (:451-469) */
    if (c->brk > 0.01) {
        double sfac = 1.0 - pymin(0.3, fabs(c->steer) * 1.5);
        double mbf = CAR_MASS * 14.0 * sfac;
        double bf = mbf * c->brk;
        double speed = f32len(w->v);
        if (speed > 0.1) {
            double dx = -(double)w->v.x / speed, dy = -(double)w->v.y / speed;
            ob_apply_force_center(w, OV(bf * dx, bf * dy));
            update_friction(c, 0.0);
        }
    }
    /* _apply_aerodynamic_drag (:471-484) */
    {
        double speed = f32len(w->v);
        if (speed > 0.1) {
            double mag = DRAG_CONSTANT * speed * speed;
            double dx = -(double)w->v.x / speed, dy = -(double)w->v.y / speed;
            ob_apply_force_center(w, OV(mag * dx, mag * dy));
        }
    }
    /* _apply_rolling_resistance (:486-500) */
    {
        double speed = f32len(w->v);
        if (speed > 0.1) {
            double rr = ROLLING_RESISTANCE_FORCE;
            double dx = -(double)w->v.x / speed, dy = -(double)w->v.y / speed;
            ob_apply_force_center(w, OV(rr * dx, rr * dy));
        }
    }
    /* _get_acceleration (:832-892) */
    double alon, alat;
    {
        double cvx = w->v.x, cvy = w->v.y;
        double ax = (cvx - c->pvx) / dt, ay = (cvy - c->pvy) / dt;
        float fwx = w->xf.q.c * 1.0f - w->xf.q.s * 0.0f, fwy = w->xf.q.s * 1.0f + w->xf.q.c * 0.0f;
        float rtx = w->xf.q.c * 0.0f - w->xf.q.s * 1.0f, rty = w->xf.q.s * 0.0f + w->xf.q.c * 1.0f;
        double lon = ax * fwx + ay * fwy, lat = ax * rtx + ay * rty;
        lon = pymax(-12.0, pymin(12.0, lon));
        lat = pymax(-12.0, pymin(12.0, lat));
        int slot = (c->acc_head + c->acc_len) % 10;
        if (c->acc_len == 10) { c->acc[c->acc_head][0] = lon; c->acc[c->acc_head][1] = lat; c->acc_head = (c->acc_head + 1) % 10; }
        else { c->acc[slot][0] = lon; c->acc[slot][1] = lat; c->acc_len++; }
        double s0 = 0.0, s1 = 0.0;
        for (int k = 0; k < c->acc_len; ++k) { int idx = (c->acc_head + k) % 10; s0 += c->acc[idx][0]; s1 += c->acc[idx][1]; }
        alon = s0 / c->acc_len; alat = s1 / c->acc_len;
        ODBG(6, alon); ODBG(7, alat);

        c->pvx = cvx; c->pvy = cvy;
    }
    /* TyreManager.update (src/tyre_manager.py:78-97) */
    {
        double speed = f32len(w->v);
        double loads[4];
        weight_transfer(c, alon, alat, speed, loads);
        double fr[4]; memcpy(fr, c->fric, sizeof fr);
        ODBG(8, fr[0]); ODBG(9, fr[2]);

        for (int i = 0; i < 4; ++i) c->load[i] = loads[i];
        for (int i = 0; i < 4; ++i) tyre_update(c, i, dt, loads[i], fr[i], speed, alat, c->slip);
    }
    /* _apply_lateral_tire_forces (:635-700) */
    {
        double speed = f32len(w->v);
        if (speed > 0.05) {
            c->lfm = 0.0; c->slip = 0.0;
            double cs = f32len(w->v);
            if (!(cs < 0.05)) {
                double fx = (double)(w->xf.q.c * 1.0f - w->xf.q.s * 0.0f), fy = (double)(w->xf.q.s * 1.0f + w->xf.q.c * 0.0f);
                double vnx = (double)w->v.x / cs, vny = (double)w->v.y / cs;
                double cr = vnx * fy - vny * fx, dt_ = vnx * fx + vny * fy;
                double sr = atan2(fabs(cr), dt_);
                c->slip = fabs(sr) * DEG_PER_RAD;
                double dvx = fx * cs, dvy = fy * cs;
                double ex = dvx - (double)w->v.x, ey = dvy - (double)w->v.y;
                double aff = CAR_MASS * 5.0;
                double cx = ex * aff, cy = ey * aff;
                double grip = total_grip(c);
                double pbf = CAR_MASS * GRAVITY_MS2 * grip * 1.0;
                double mf = pymin(30000.0 * grip, pbf);
                double fm = pow(P2(cx) + P2(cy), 0.5);
                ODBG(10, cs); ODBG(11, cx); ODBG(12, cy); ODBG(13, fm); ODBG(14, c->slip);

                if (fm > mf) { double sc = mf / fm; cx = cx * sc; cy = cy * sc; fm = mf; }
                c->lfm = fm;
                ob_apply_force_center(w, OV(cx, cy));
            }
        }
    }
    /* _apply_angular_damping (:502-507) */
    ODBG(15, w->force.x); ODBG(16, w->force.y); ODBG(17, w->torque);

    ob_apply_torque(w, (float)(-(double)w->w * CAR_MASS * 4.0));
    /* _apply_banking_forces (:509-566); the lateral assist per segment is host-precomputed
       in the product, here it is evaluated as the reference does */
    if (!(fabs(c->bank) < 0.1)) {
        double speed = f32len(w->v);
        if (!(speed < 1.0)) {
            double br = c->bank * RAD_PER_DEG;
            double gc = CAR_MASS * 9.81;
            double nfg = gc * sin(fabs(br));
            double la = nfg * 0.3;
            if (!(fabs(la) < 1.0) && speed > 5.0) {
                double vx = (double)w->v.x / speed, vy = (double)w->v.y / speed;
                double fdx = -vy, fdy = vx;
                double sg = copysign(1.0, c->bank);
                ob_apply_force_center(w, OV(fdx * la * sg, fdy * la * sg));
            }
        }
    }
    /* _apply_steering_torque (:568-584) */
    if (fabs(c->steer) > 0.01) {
        double speed = f32len(w->v);
        if (speed > 0.1) {
            double dav = speed * tan(c->steer) / CAR_WHEELBASE;
            double err = dav - (double)w->w;
            ob_apply_torque(w, (float)(err * CAR_MASS * 0.8));
        }
    }
    /* the end-of-update friction rewrite (:375-382) is overwritten before its next
       read (the next _apply_engine_force) -> dead for every output; omitted. */
}

/* CarPhysics.get_banking_angle_at_position (src/car_physics.py:631-672) */
static double banking_at(const otrack *t, double px, double py) {
    double best = INFINITY; int bi = -1;
    for (int k = 0; k < t->nseg; ++k) {
        const oseg *s = &t->seg[k];
        double ll = P2(s->ex - s->sx) + P2(s->ey - s->sy), d;
        if (ll == 0) d = sqrt(P2(px - s->sx) + P2(py - s->sy));
        else {
            double tt = ((px - s->sx) * (s->ex - s->sx) + (py - s->sy) * (s->ey - s->sy)) / ll;
            tt = pymax(0, pymin(1, tt));
            double qx = s->sx + tt * (s->ex - s->sx), qy = s->sy + tt * (s->ey - s->sy);
            d = sqrt(P2(px - qx) + P2(py - qy));
        }
        if (d < best) { best = d; bi = k; }
    }
    return bi >= 0 ? t->seg[bi].banking : 0.0;
}

/* CarEnv._calculate_track_progress (src/car_env.py:1544-1611) */
static double track_progress(const otrack *t, double px, double py) {
    double best = INFINITY; int bi = 0; double bx = 0, by = 0;
    for (int k = 0; k < t->nseg; ++k) {
        const oseg *s = &t->seg[k];
        double dx = s->ex - s->sx, dy = s->ey - s->sy, ll = dx * dx + dy * dy, qx, qy;
        if (ll < 1e-6) { qx = s->sx; qy = s->sy; }
        else {
            double tt = pymax(0, pymin(1, ((px - s->sx) * dx + (py - s->sy) * dy) / ll));
            qx = s->sx + tt * dx; qy = s->sy + tt * dy;
        }
        double d2 = P2(px - qx) + P2(py - qy);
        if (d2 < best) { best = d2; bi = k; bx = qx; by = qy; }
    }
    double tot = 0.0;
    for (int k = 0; k < bi; ++k) {
        const oseg *s = &t->seg[k];
        tot += sqrt(P2(s->ex - s->sx) + P2(s->ey - s->sy));
    }
    const oseg *s = &t->seg[bi];
    tot += sqrt(P2(bx - s->sx) + P2(by - s->sy));
    return tot;
}

/* LapTimer._is_position_on_startline (src/lap_timer.py:205-242) */
static int on_startline(const otrack *t, double px, double py) {
    const oseg *s = &t->seg[t->startline];
    double dx = s->ex - s->sx, dy = s->ey - s->sy, ll = dx * dx + dy * dy, d;
    if (ll < 1e-6) d = sqrt(P2(px - s->sx) + P2(py - s->sy));
    else {
        double tt = pymax(0, pymin(1, ((px - s->sx) * dx + (py - s->sy) * dy) / ll));
        double qx = s->sx + tt * dx, qy = s->sy + tt * dy;
        d = sqrt(P2(px - qx) + P2(py - qy));
    }
    return d <= (s->width / 2.0);
}
/* LapTimer.update (src/lap_timer.py:95-203, 244-272); returns lap completed */
static int lap_update(const otrack *t, ocar *c, double px, double py, double sim) {
    if (c->lt_timing) c->lt_cur = sim - c->lt_start;
    if (c->lt_has_pos) {
        double dx = px - c->lt_px, dy = py - c->lt_py, d = sqrt(dx * dx + dy * dy);
        if (d < 50.0) c->lt_dist += d;
    }
    int done = 0;
    if (t->startline >= 0 && c->lt_has_pos) {
        int now = on_startline(t, px, py), before = on_startline(t, c->lt_px, c->lt_py);
        if (now && !before) {
            if (c->lt_crossed && c->lt_timing) {
                /* the 2 s cooldown compares time.time() with a sim-time stamp: never fires */
                double minlap = t->total_length > 0 ? t->total_length * 0.95 : 100.0;
                if (c->lt_cur < 10.0) {}
                else if (c->lt_dist < minlap) {}
                else {
                    double ct = c->lt_cur;
                    c->lt_last = ct; c->lt_has_last = 1;
                    if (!c->lt_has_best || ct < c->lt_best) { c->lt_best = ct; c->lt_has_best = 1; }
                    c->lt_start = sim; c->lt_cur = 0.0; c->lt_timing = 1;
                    c->lt_laps += 1; c->lt_dist = 0.0;
                    done = 1;
                }
            } else if (!c->lt_crossed) {
                c->lt_crossed = 1; c->lt_timing = 1; c->lt_start = sim; c->lt_cur = 0.0; c->lt_dist = 0.0;
            }
        }
    }
    c->lt_px = px; c->lt_py = py; c->lt_has_pos = 1;
    return done;
}

/* ---------------- env ------------------------------------------------------- */
static void car_fresh(oenv *e, ocar *c) {
    memset(c, 0, sizeof(*c));
    c->W = &e->trk.W;
    ov2 p = OV(e->start_x, e->start_y);
    ob_world_init(&c->w, &e->trk.W, p, (float)e->start_angle);
    c->rpm = 1000.0;
    for (int i = 0; i < 4; ++i) { c->temp[i] = 80.0; c->wear[i] = 0.0; c->load[i] = (CAR_MASS * GRAVITY_MS2 * 0.5) / 2.0; }
}
/* CarPhysics.reset_car + Car.reset (src/car_physics.py:550-571, src/car.py:1027-1058) */
static void car_reset(oenv *e, ocar *c) {
    oworld *w = &c->w; const owalls *W = &e->trk.W;
    ov2 p = OV(e->start_x, e->start_y); float a = (float)e->start_angle;
    ob_set_transform(w, W, p, w->a);          /* body.position = position */
    ob_set_transform(w, W, w->xf.p, a);       /* body.angle = angle */
    ob_set_transform(w, W, p, w->a);          /* Car.reset: body.position */
    ob_set_transform(w, W, w->xf.p, a);       /*            body.angle */
    w->v.x = 0.0f; w->v.y = 0.0f; w->w = 0.0f;   /* zero setters do not wake */
    c->thr_in = c->brk_in = c->str_in = 0.0; c->thr = c->brk = c->steer = 0.0;
    c->rpm = 1000.0;
    for (int i = 0; i < 4; ++i) { c->temp[i] = 80.0; c->wear[i] = 0.0; c->load[i] = (CAR_MASS * GRAVITY_MS2 * 0.5) / 2.0; c->fric[i] = 0.0; }
    c->pvx = c->pvy = 0.0; c->acc_len = 0; c->acc_head = 0; c->lfm = 0.0; c->slip = 0.0;
    /* current_banking_angle is NOT reset (src/car.py:1027-1058) */
    c->nact = 0; c->imp_present = 0; c->imp = 0.0;
}

static void collision_data(const ocar *c, double *imp, double *ang) {
    double ci = c->imp_present ? c->imp : 0.0;
    *imp = 0.0; *ang = 0.0;
    if (ci < 100.0) return;
    *imp = ci;
    if (c->nact > 0) {
        double na = atan2((double)c->act_ny[0], (double)c->act_nx[0]);
        double a = na - (double)c->w.a;
        while (a > PI_) a -= 2 * PI_;
        while (a < -PI_) a += 2 * PI_;
        *ang = a;
    }
}

/* DistanceSensor.get_sensor_distances (src/distance_sensor.py:71-117) of a car at p1 with body angle ang, as
   _get_multi_obs stores them (src/car_env.py:946): 16 rays 22.5 deg apart, 250 m, b2World.RayCast closest hit */
static void sensors16(const oenv *e, ov2 p1, double ang, float *out) {
    const double px = p1.x, py = p1.y;
    for (int i = 0; i < 16; ++i) {
        double sa = -((double)i * (360.0 / 16) * RAD_PER_DEG) + ang;
        double dx = cos(sa), dy = sin(sa);
        ov2 p2 = OV(px + dx * 250.0, py + dy * 250.0);
        float fr = ob_raycast(&e->trk.W, p1, p2);
        double hd = fr >= 0.0f ? (double)fr * 250.0 : 250.0;
        float d32 = (float)hd;
        float v = d32 / 250.0f;
        out[i] = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
    }
}

/* CarEnv._get_multi_obs for one car (src/car_env.py:891-956) */
static void car_obs(oenv *e, ocar *c, float *o) {
    const oworld *w = &c->w;
    double px = w->xf.p.x, py = w->xf.p.y, vx = w->v.x, vy = w->v.y, ang = w->a, av = w->w;
    o[0] = (float)npclip(px / 10000.0, -1, 1); o[1] = (float)npclip(py / 10000.0, -1, 1);
    o[2] = (float)npclip(vx / 111.1, -1, 1); o[3] = (float)npclip(vy / 111.1, -1, 1);
    double sm = pow(P2(vx) + P2(vy), 0.5);
    o[4] = (float)npclip(sm / 111.1, 0, 1);
    o[5] = (float)npclip(ang / PI_, -1, 1); o[6] = (float)npclip(av / 10.0, -1, 1);
    for (int i = 0; i < 4; ++i) {
        o[7 + i] = (float)npclip(c->load[i] / MAX_TYRE_LOAD, 0, 1);
        o[11 + i] = (float)npclip(c->temp[i] / 200.0, 0, 1);
        o[15 + i] = (float)npclip(c->wear[i] / 100.0, 0, 1);
    }
    double imp, ca; collision_data(c, &imp, &ca);
    o[19] = (float)npclip(imp / 50000.0, 0, 1); o[20] = (float)npclip(ca / PI_, -1, 1);
    o[21] = (float)npclip(c->cum_impact / 250000.0, 0, 1);
    sensors16(e, w->xf.p, ang, o + 22);
}

static int all_active_completed(oenv *e, int env) {
    int any = 0;
    for (int k = 0; k < e->C; ++k) {
        ocar *c = &e->car[env * e->C + k];
        if (c->disabled) continue;
        any = 1;
        if (c->lt_laps < 1) return 0;
    }
    return any;
}

static void env_reset(oenv *e, int env) {
    for (int k = 0; k < e->C; ++k) {
        ocar *c = &e->car[env * e->C + k];
        if (!e->created[env]) car_fresh(e, c);
        else car_reset(e, c);
        olistener L = { c, lis_begin, lis_end, lis_post };
        (void)L;
        c->lt_timing = 0; c->lt_start = 0; c->lt_cur = 0.0; c->lt_has_last = c->lt_has_best = 0;
        c->lt_crossed = 0; c->lt_has_pos = 0; c->lt_laps = 0; c->lt_dist = 0.0;
        c->disabled = 0; c->just_disabled = 0; c->cum_impact = 0.0;
        c->stuck_dur = 0.0; c->has_stuck_start = 0;
        c->prev_px = c->w.xf.p.x; c->prev_py = c->w.xf.p.y;
        c->back = c->prev_back = 0.0; c->first_step = 1; c->prev_laps = 0; c->cum_reward = 0.0f; c->cum_reward_info = 0.0f;
        c->prog_hist = track_progress(&e->trk, c->w.xf.p.x, c->w.xf.p.y);
    }
    e->created[env] = 1;
    e->sim_time[env] = 0.0; e->pending[env] = 0; e->term_reason[env] = 0;
    e->terminated[env] = 0; e->truncated[env] = 0;
    for (int k = 0; k < e->C; ++k) { ocar *c = &e->car[env * e->C + k]; car_obs(e, c, c->obs); c->reward = 0.0f; }
}

/* CarEnv._step_multi_car (src/car_env.py:723-803) for one env; act: C x 3 internal f32 */
static void env_step(oenv *e, int env, const float *act) {
    const double dt = PHYS_DT;
    const otrack *t = &e->trk;
    int C = e->C;
    /* update_physics (:537-573) */
    for (int k = 0; k < C; ++k) {
        ocar *c = &e->car[env * C + k];
        float a0 = act[k * 3 + 0], a1 = act[k * 3 + 1], a2 = act[k * 3 + 2];
        if (c->disabled) { a0 = 0.0f; a1 = 0.0f; a2 = 0.0f; }
        /* CarPhysics.step (src/car_physics.py:341-384) */
        c->thr_in = pymax(0.0, pymin(1.0, (double)a0));
        c->brk_in = pymax(0.0, pymin(1.0, (double)a1));
        c->str_in = pymax(-1.0, pymin(1.0, (double)a2));
        g_cur_car = env * C + k;
        car_update_physics(c, dt);
        g_cur_car = -2;
        olistener L = { c, lis_begin, lis_end, lis_post };
        ob_step(&c->w, &t->W, &L, (float)dt, 6, 4);
        if (t->has_banking) c->bank = banking_at(t, c->w.xf.p.x, c->w.xf.p.y);
        else c->bank = 0.0;
        /* _run_single_physics_step (src/car_env.py:575-676) */
        if (!c->disabled) {
            double imp = c->imp_present ? c->imp : 0.0;
            if (imp > 50000.0) { c->disabled = 1; c->just_disabled = 1; }
            if (imp > 100.0) c->cum_impact += imp;
            if (c->cum_impact > 250000.0 && !c->disabled) { c->disabled = 1; c->just_disabled = 1; }
            double speed = f32len(c->w.v);
            if (speed < 0.5) c->stuck_dur = c->stuck_dur + dt;
            else { c->stuck_dur = 0.0; c->has_stuck_start = 0; }
        }
        int lap = lap_update(t, c, c->w.xf.p.x, c->w.xf.p.y, e->sim_time[env]);
        if (lap && e->reset_on_lap && all_active_completed(e, env)) e->pending[env] = 1;
    }
    e->sim_time[env] += dt;
    /* _check_and_disable_cars (:805-888) */
    for (int k = 0; k < C; ++k) {
        ocar *c = &e->car[env * C + k];
        if (c->disabled) continue;
        double speed = f32len(c->w.v);
        if (speed < 0.5 && c->stuck_dur > 0) {
            double px = c->w.xf.p.x, py = c->w.xf.p.y;
            if (!c->has_stuck_start) { c->has_stuck_start = 1; c->stuck_sx = px; c->stuck_sy = py; }
            double dx = px - c->stuck_sx, dy = py - c->stuck_sy;
            double moved = pow(P2(dx) + P2(dy), 0.5);
            if (c->stuck_dur > 10.0) {
                int dis = 0;
                if (moved < 1.0) dis = 1;
                else if (c->stuck_dur > 15.0) dis = 1;
                if (dis) { c->disabled = 1; c->just_disabled = 1; }
            }
        } else { c->stuck_dur = 0.0; c->has_stuck_start = 0; }
    }
    /* observations (:891-956) */
    for (int k = 0; k < C; ++k) { ocar *c = &e->car[env * C + k]; car_obs(e, c, c->obs); }
    /* rewards (:980-1113) */
    for (int k = 0; k < C; ++k) {
        ocar *c = &e->car[env * C + k];
        if (c->disabled && !c->just_disabled) { c->reward = 0.0f; continue; }
        double r = c->just_disabled ? 10.0 : 0.0;
        if (!c->disabled) r -= 0.05;
        if (!c->disabled) { double imp = c->imp_present ? c->imp : 0.0; if (fabs(imp) > 0) r -= 0.5; }
        double px = c->w.xf.p.x, py = c->w.xf.p.y;
        double dx = px - c->prev_px, dy = py - c->prev_py;
        r += pow(P2(dx) + P2(dy), 0.5) * 0.15;
        c->prev_px = px; c->prev_py = py;
        if (!c->first_step) {
            double prog = track_progress(t, px, py);
            double L = t->total_length, pd = prog - c->prog_hist;
            if (pd > L / 2) pd -= L; else if (pd < -L / 2) pd += L;
            if (pd < 0) {
                c->back += fabs(pd);
                if (c->back > 200.0 && !c->disabled) { c->disabled = 1; c->just_disabled = 1; }
                if (c->back > 25.0) {
                    double ce = pymax(0, c->back - 25.0), pe = pymax(0, c->prev_back - 25.0);
                    double nb = ce - pe;
                    if (nb > 0) r -= nb * 0.05;
                }
            } else { c->back = 0.0; c->prev_back = 0.0; }
            c->prog_hist = prog;
        } else {
            c->prog_hist = track_progress(t, px, py);
            c->first_step = 0;
        }
        if (c->lt_laps > c->prev_laps) { r += 0.0 * (c->lt_laps - c->prev_laps); c->prev_laps = c->lt_laps; }
        if (!c->disabled) c->prev_back = c->back;
        c->reward = (float)r;
    }
    /* termination (:1115-1158) uses cumulative rewards BEFORE this step */
    int term = 0, trunc = 0, ndis = 0, active = 0, below = 0;
    for (int k = 0; k < C; ++k) { ocar *c = &e->car[env * C + k]; ndis += c->disabled; }
    if (ndis >= C) { term = 1; e->term_reason[env] = 1; }
    else {
        for (int k = 0; k < C; ++k) { ocar *c = &e->car[env * C + k]; if (!c->disabled) { active++; if (c->cum_reward < -250.0f) below++; } }
        if (active > 0 && below == active) { term = 1; e->term_reason[env] = 2; }
        else if (e->reset_on_lap && e->sim_time[env] > 60.0) { term = 1; e->term_reason[env] = 3; }
        else if (e->sim_time[env] > 180.0) { trunc = 1; e->term_reason[env] = 4; }
    }
    for (int k = 0; k < C; ++k) {
        ocar *c = &e->car[env * C + k];
        c->imp_at_obs = c->imp_present ? c->imp : 0.0;
        c->cum_reward_info = c->cum_reward;             /* info is built before the update */
        c->imp = 0.0; c->imp_present = 1;               /* (:775-779) */
        c->cum_reward = c->cum_reward + c->reward;      /* float32 accumulation (NEP 50) */
    }
    if (e->pending[env]) { e->pending[env] = 0; term = 1; }
    for (int k = 0; k < C; ++k) e->car[env * C + k].just_disabled = 0;
    e->terminated[env] = term; e->truncated[env] = trunc;
}

/* ================= exported ctypes API (tests / bench cpu_baseline only) ===== */
EXPORT void *or_create(const char *track_path, int E, int C, int reset_on_lap) {
    oenv *e = calloc(1, sizeof(oenv));
    if (load_track(&e->trk, track_path, e->err, sizeof e->err) != 0) { fprintf(stderr, "%s\n", e->err); free(e); return NULL; }
    build_walls(&e->trk);
    e->E = E; e->C = C; e->reset_on_lap = reset_on_lap;
    e->start_x = e->trk.start_x; e->start_y = e->trk.start_y; e->start_angle = 0.0;
    e->car = calloc((size_t)E * C, sizeof(ocar));
    e->sim_time = calloc((size_t)E, sizeof(double));
    e->created = calloc((size_t)E, sizeof(int)); e->pending = calloc((size_t)E, sizeof(int));
    e->term_reason = calloc((size_t)E, sizeof(int)); e->terminated = calloc((size_t)E, sizeof(int));
    e->truncated = calloc((size_t)E, sizeof(int));
    return e;
}
/* CarEnv(start_position=..., start_angle=...) (src/car_env.py:82-83,114-115): the pose Car() and
   CarPhysics.reset_car use for every car (src/car_env.py:391,398); the default is the track's first
   GRID/STARTLINE segment start (src/car_env.py:236-241) and angle 0. */
EXPORT void or_set_start(void *h, double x, double y, double angle) {
    oenv *e = h; e->start_x = x; e->start_y = y; e->start_angle = angle;
}
EXPORT void or_destroy(void *h) {
    oenv *e = h; if (!e) return;
    free(e->car); free(e->sim_time); free(e->created); free(e->pending); free(e->term_reason);
    free(e->terminated); free(e->truncated); free(e);
}
EXPORT int or_num_walls(void *h) { return ((oenv *)h)->trk.W.n; }
EXPORT int or_num_segments(void *h) { return ((oenv *)h)->trk.nseg; }
EXPORT double or_total_length(void *h) { return ((oenv *)h)->trk.total_length; }
/* walls as double [cx, cy, angle, half_len] (pre float cast) and float [px,py,angle,hx,hy,s,c,lox,loy,hix,hiy,key] */
EXPORT void or_walls(void *h, double *dbl, float *flt) {
    oenv *e = h; otrack *t = &e->trk;
    for (int j = 0; j < t->W.n; ++j) {
        if (dbl) { dbl[j * 4 + 0] = t->wall_cx[j]; dbl[j * 4 + 1] = t->wall_cy[j]; dbl[j * 4 + 2] = t->wall_ang[j]; dbl[j * 4 + 3] = t->wall_hl[j]; }
        if (flt) {
            float *f = flt + j * 12;
            f[0] = t->W.p[j].x; f[1] = t->W.p[j].y; f[2] = t->W.angle[j]; f[3] = t->W.hx[j]; f[4] = t->W.hy[j];
            f[5] = t->W.q[j].s; f[6] = t->W.q[j].c; f[7] = t->W.fat[j].lo.x; f[8] = t->W.fat[j].lo.y;
            f[9] = t->W.fat[j].hi.x; f[10] = t->W.fat[j].hi.y; f[11] = (float)t->W.key[j];
        }
    }
}
/* segments as double [type, length, sx, sy, ex, ey, width, curve_angle, curve_radius, left, start_heading, end_heading, banking] */
EXPORT void or_segments(void *h, double *out) {
    otrack *t = &((oenv *)h)->trk;
    for (int k = 0; k < t->nseg; ++k) {
        const oseg *s = &t->seg[k]; double *o = out + k * 13;
        o[0] = s->type; o[1] = s->length; o[2] = s->sx; o[3] = s->sy; o[4] = s->ex; o[5] = s->ey; o[6] = s->width;
        o[7] = s->curve_angle; o[8] = s->curve_radius; o[9] = s->dir_left; o[10] = s->start_heading; o[11] = s->end_heading; o[12] = s->banking;
    }
}
EXPORT void or_reset(void *h, int env) { env_reset((oenv *)h, env); }
/* actions: E*C*2 float32 [throttle_brake, steering] (BaseEnv._convert_to_internal_action) */
EXPORT void or_step(void *h, const float *actions2) {
    oenv *e = h;
    float *act = malloc(sizeof(float) * 3 * (size_t)e->C);
    for (int env = 0; env < e->E; ++env) {
        for (int k = 0; k < e->C; ++k) {
            float tb = actions2[(env * e->C + k) * 2 + 0], st = actions2[(env * e->C + k) * 2 + 1];
            if (tb >= 0) { act[k * 3 + 0] = tb; act[k * 3 + 1] = 0.0f; }
            else { act[k * 3 + 0] = 0.0f; act[k * 3 + 1] = -tb; }
            act[k * 3 + 2] = st;
        }
        env_step(e, env, act);
    }
    free(act);
}
/* copy outputs: obs E*C*38, reward E*C, flags E*C (bit0 disabled), env E*3 (terminated, truncated, reason) */
EXPORT void or_outputs(void *h, float *obs, float *rew, uint8_t *cflags, int32_t *eflags) {
    oenv *e = h;
    for (int i = 0; i < e->E * e->C; ++i) {
        ocar *c = &e->car[i];
        if (obs) memcpy(obs + i * 38, c->obs, sizeof(float) * 38);
        if (rew) rew[i] = c->reward;
        /* bit 0 disabled, bit 2 collision impulse at this step's observation (nascar.h car_flags) */
        if (cflags) cflags[i] = (uint8_t)((c->disabled ? 1 : 0) | (c->imp_at_obs != 0.0 ? 4 : 0));
    }
    if (eflags) for (int env = 0; env < e->E; ++env) { eflags[env * 3] = e->terminated[env]; eflags[env * 3 + 1] = e->truncated[env]; eflags[env * 3 + 2] = e->term_reason[env]; }
}
/* per-car info vector (doubles): see tests/oracle_lib.py ORACLE_INFO_FIELDS */
EXPORT void or_car_info(void *h, int idx, double *o) {
    oenv *e = h; ocar *c = &e->car[idx]; int env = idx / e->C;
    o[0] = c->w.xf.p.x; o[1] = c->w.xf.p.y; o[2] = c->w.v.x; o[3] = c->w.v.y; o[4] = c->w.a; o[5] = c->w.w;
    o[6] = c->rpm; o[7] = c->lfm; o[8] = c->slip; o[9] = c->bank;
    for (int i = 0; i < 4; ++i) { o[10 + i] = c->load[i]; o[14 + i] = c->temp[i]; o[18 + i] = c->wear[i]; }
    o[22] = c->lt_laps; o[23] = c->lt_has_last ? c->lt_last : NAN; o[24] = c->lt_has_best ? c->lt_best : NAN;
    o[25] = c->lt_timing; o[26] = c->lt_cur; o[27] = c->lt_dist;
    o[28] = c->disabled; o[29] = c->cum_impact; o[30] = c->cum_reward; o[31] = c->stuck_dur;
    o[32] = c->back; o[33] = c->prog_hist; o[34] = e->sim_time[env]; o[35] = c->imp_at_obs;
    o[36] = c->w.sleepTime; o[37] = c->w.awake; o[38] = c->w.nct; o[39] = c->w.overflow;
    o[40] = ob_query_on_wall(&e->trk.W, c->w.xf.p.x, c->w.xf.p.y, 0.5) ? 0.0 : 1.0;   /* on_track */
    o[41] = c->nact;
    o[42] = c->cum_reward_info;
    o[43] = (double)sqrtf(c->w.v.x * c->w.v.x + c->w.v.y * c->w.v.y);   /* car_speed_ms */
}
/* unit hooks */
EXPORT float or_sinf(float x) { return ob_sinf(x); }
EXPORT float or_cosf(float x) { return ob_cosf(x); }
/* the 16 sensor values of n arbitrary poses [n][3] (x, y, angle) float32 -> out [n][16] (sensor parity tests) */
EXPORT void or_sensors(void *h, const float *poses, int n, float *out) {
    const oenv *e = h;
    for (int k = 0; k < n; ++k)
        sensors16(e, OV(poses[3 * k], poses[3 * k + 1]), (double)poses[3 * k + 2], out + 16 * (size_t)k);
}
EXPORT float or_raycast(void *h, float x1, float y1, float x2, float y2) {
    ov2 a = { x1, y1 }, b = { x2, y2 };
    return ob_raycast(&((oenv *)h)->trk.W, a, b);
}
/* state injection for unit tests of the vehicle model: set body state of a car */
EXPORT void or_set_body(void *h, int idx, float x, float y, float a, float vx, float vy, float w) {
    oenv *e = h; ocar *c = &e->car[idx];
    c->w.c.x = x; c->w.c.y = y; c->w.a = a; c->w.v.x = vx; c->w.v.y = vy; c->w.w = w;
    ob_rot_set(&c->w.xf.q, a); c->w.xf.p = c->w.c;
}

/* ================= hybrid hooks: a bare Box2D world per car for gen_golden.py =====
 * gen_golden.py runs the REFERENCE's own Python CarEnv with a fake `Box2D` module
 * whose worlds are these (so the reference's car model, tyres, lap timer, rewards,
 * disable/termination and obs code run unchanged on top of b2_oracle.c). */
typedef void (*hb_begin_t)(int wall, float nx, float ny);
typedef void (*hb_end_t)(int wall);
typedef void (*hb_post_t)(int count, float n0, float n1);
typedef struct { hb_begin_t b; hb_end_t e; hb_post_t p; } hbcb;
static void hb_lb(void *u, int wall, ov2 n) { ((hbcb *)u)->b(wall, n.x, n.y); }
static void hb_le(void *u, int wall) { ((hbcb *)u)->e(wall); }
static void hb_lp(void *u, int count, const float *ni) { ((hbcb *)u)->p(count, ni[0], count > 1 ? ni[1] : 0.0f); }

EXPORT void *hb_world_create(void *h, float x, float y, float angle) {
    oenv *e = h; oworld *w = calloc(1, sizeof(oworld));
    ov2 p = { x, y };
    ob_world_init(w, &e->trk.W, p, angle);
    return w;
}
EXPORT void hb_world_destroy(void *w) { free(w); }
EXPORT void hb_apply_force(void *w, float fx, float fy, float px, float py) { ov2 f = { fx, fy }, p = { px, py }; ob_apply_force(w, f, p); }
EXPORT void hb_apply_force_center(void *w, float fx, float fy) { ov2 f = { fx, fy }; ob_apply_force_center(w, f); }
EXPORT void hb_apply_torque(void *w, float t) { ob_apply_torque(w, t); }
EXPORT void hb_step(void *h, void *w, float dt, int vi, int pi, hb_begin_t b, hb_end_t en, hb_post_t p) {
    oenv *e = h; hbcb cb = { b, en, p };
    olistener L = { &cb, hb_lb, hb_le, hb_lp };
    ob_step(w, &e->trk.W, &L, dt, vi, pi);
}
/* state: [p.x, p.y, angle(sweep a), v.x, v.y, w, q.s, q.c] */
EXPORT void hb_get(void *w_, float *o) {
    oworld *w = w_;
    o[0] = w->xf.p.x; o[1] = w->xf.p.y; o[2] = w->a; o[3] = w->v.x; o[4] = w->v.y; o[5] = w->w; o[6] = w->xf.q.s; o[7] = w->xf.q.c;
}
EXPORT void hb_set_transform(void *h, void *w, float x, float y, float a) { ov2 p = { x, y }; ob_set_transform(w, &((oenv *)h)->trk.W, p, a); }
EXPORT void hb_set_velocity(void *w_, float vx, float vy) {
    oworld *w = w_;
    if (vx * vx + vy * vy > 0.0f) { if (!w->awake) { w->awake = 1; w->sleepTime = 0.0f; } }
    w->v.x = vx; w->v.y = vy;
}
EXPORT void hb_set_angular_velocity(void *w_, float av) {
    oworld *w = w_;
    if (av * av > 0.0f) { if (!w->awake) { w->awake = 1; w->sleepTime = 0.0f; } }
    w->w = av;
}

/* full per-car state in the GPU arena field order (tests/gpu_state.py F32, F64, I32 lists) */
EXPORT void or_car_state(void *h, int idx, double *o) {
    oenv *e = h; ocar *c = &e->car[idx]; oworld *w = &c->w;
    double v[] = {
        w->c.x, w->c.y, w->a, w->v.x, w->v.y, w->w, w->xf.q.s, w->xf.q.c, w->xf.p.x, w->xf.p.y, w->sleepTime, w->inv_dt0,
        w->fat.lo.x, w->fat.lo.y, w->fat.hi.x, w->fat.hi.y, c->cum_reward, c->cum_reward_info,
        c->rpm, c->pvx, c->pvy, c->lfm, c->slip, c->bank, c->load[0], c->load[1], c->load[2], c->load[3],
        c->temp[0], c->temp[1], c->temp[2], c->temp[3], c->wear[0], c->wear[1], c->wear[2], c->wear[3], c->imp,
        c->lt_start, c->lt_cur, c->lt_last, c->lt_best, c->lt_px, c->lt_py, c->lt_dist, c->cum_impact, c->stuck_dur,
        c->stuck_sx, c->stuck_sy, c->prev_px, c->prev_py, c->prog_hist, c->back, c->prev_back, c->imp_at_obs,
        w->awake, w->nct, w->overflow, c->acc_len, c->acc_head, c->imp_present, c->nact, c->lt_timing, c->lt_has_last,
        c->lt_has_best, c->lt_crossed, c->lt_has_pos, c->lt_laps, c->disabled, c->has_stuck_start, c->first_step, c->prev_laps };
    memcpy(o, v, sizeof v);
}

/* ================= state injection (test infrastructure) ==========================
 * The inverse of or_car_state: a car's full state in the GPU arena's layout (nascar_layout.h) -- the f32 / f64 /
 * i32 per-car fields in their field order, the 10-sample acceleration ring (acc[slot][lon, lat], slot = acc_head +
 * k oldest first, as here), the b2Contact records (MAXC x 20 words of nascar::DContact) and the listener's
 * active-contact keys / first normals -- so the oracle can continue from a state the GPU reached (a steady state
 * the CPU cannot afford to settle to).  Transient b2Body fields (force, torque, sweep c0 / a0 / alpha0, the proxy
 * move flag) are zero / equal to the body at a step boundary, as on the GPU. */
#define GPU_MAXC 16
EXPORT void or_set_car_full(void *h, int idx, const double *f32v, const double *f64v, const int *i32v,
                            const double *acc20, const int32_t *ct_words, const int32_t *act_key, const float *act_n) {
    oenv *e = h; ocar *c = &e->car[idx]; oworld *w = &c->w;
    w->c.x = (float)f32v[0]; w->c.y = (float)f32v[1]; w->a = (float)f32v[2];
    w->v.x = (float)f32v[3]; w->v.y = (float)f32v[4]; w->w = (float)f32v[5];
    w->xf.q.s = (float)f32v[6]; w->xf.q.c = (float)f32v[7]; w->xf.p.x = (float)f32v[8]; w->xf.p.y = (float)f32v[9];
    w->sleepTime = (float)f32v[10]; w->inv_dt0 = (float)f32v[11];
    w->fat.lo.x = (float)f32v[12]; w->fat.lo.y = (float)f32v[13]; w->fat.hi.x = (float)f32v[14]; w->fat.hi.y = (float)f32v[15];
    c->cum_reward = (float)f32v[16]; c->cum_reward_info = (float)f32v[17];
    w->force.x = w->force.y = 0.0f; w->torque = 0.0f;
    w->c0 = w->c; w->a0 = w->a; w->alpha0 = 0.0f; w->moved = 0;
    const double *d = f64v;
    c->rpm = d[0]; c->pvx = d[1]; c->pvy = d[2]; c->lfm = d[3]; c->slip = d[4]; c->bank = d[5];
    for (int k = 0; k < 4; ++k) { c->load[k] = d[6 + k]; c->temp[k] = d[10 + k]; c->wear[k] = d[14 + k]; }
    c->imp = d[18];
    c->lt_start = d[19]; c->lt_cur = d[20]; c->lt_last = d[21]; c->lt_best = d[22]; c->lt_px = d[23]; c->lt_py = d[24];
    c->lt_dist = d[25]; c->cum_impact = d[26]; c->stuck_dur = d[27]; c->stuck_sx = d[28]; c->stuck_sy = d[29];
    c->prev_px = d[30]; c->prev_py = d[31]; c->prog_hist = d[32]; c->back = d[33]; c->prev_back = d[34]; c->imp_at_obs = d[35];
    const int *v = i32v;
    w->awake = v[0]; w->nct = v[1]; w->overflow = v[2]; c->acc_len = v[3]; c->acc_head = v[4]; c->imp_present = v[5];
    c->nact = v[6]; c->lt_timing = v[7]; c->lt_has_last = v[8]; c->lt_has_best = v[9]; c->lt_crossed = v[10];
    c->lt_has_pos = v[11]; c->lt_laps = v[12]; c->disabled = v[13]; c->has_stuck_start = v[14]; c->first_step = v[15];
    c->prev_laps = v[16];
    c->just_disabled = 0;
    for (int s = 0; s < 10; ++s) { c->acc[s][0] = acc20[2 * s]; c->acc[s][1] = acc20[2 * s + 1]; }
    for (int i = 0; i < OB_MAXC; ++i) memset(&w->ct[i], 0, sizeof w->ct[i]);
    for (int i = 0; i < GPU_MAXC; ++i) {   /* the GPU keeps MAXC = 16 records per car (nascar_layout.h) */
        const int32_t *q = ct_words + 20 * i;
        ocontact *o = &w->ct[i];
        o->wall = q[0]; o->flags = q[1]; o->m.type = q[2]; o->m.pointCount = q[3];
        memcpy(&o->m.localNormal.x, &q[4], 4); memcpy(&o->m.localNormal.y, &q[5], 4);
        memcpy(&o->m.localPoint.x, &q[6], 4); memcpy(&o->m.localPoint.y, &q[7], 4);
        for (int p = 0; p < 2; ++p) {
            const int32_t *pp = q + 8 + 5 * p;
            memcpy(&o->m.pts[p].localPoint.x, &pp[0], 4); memcpy(&o->m.pts[p].localPoint.y, &pp[1], 4);
            memcpy(&o->m.pts[p].normalImpulse, &pp[2], 4); memcpy(&o->m.pts[p].tangentImpulse, &pp[3], 4);
            memcpy(&o->m.pts[p].id, &pp[4], 4);
        }
        memcpy(&o->toi, &q[18], 4); o->toiCount = q[19];
    }
    for (int i = 0; i < GPU_MAXC; ++i) { c->act_key[i] = act_key[i]; c->act_nx[i] = act_n[2 * i]; c->act_ny[i] = act_n[2 * i + 1]; }
}
/* per-env words of the GPU arena: simulated time, created / pending / reason / terminated / truncated */
EXPORT void or_set_env_full(void *h, int env, double sim_time, int created, int pending, int reason, int term, int trunc) {
    oenv *e = h;
    e->sim_time[env] = sim_time; e->created[env] = created; e->pending[env] = pending;
    e->term_reason[env] = reason; e->terminated[env] = term; e->truncated[env] = trunc;
}
