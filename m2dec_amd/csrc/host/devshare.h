/* devshare.c: the device-wide workgroup budget shared by every process decoding on one GPU */
#ifndef M2DEC_DEVSHARE_H
#define M2DEC_DEVSHARE_H
#ifdef __cplusplus
extern "C" {
#endif

/* units per CU: divisible by every resident-workgroups-per-CU count 1..6, so a workgroup's cost
 * (units per CU / resident per CU) is exact for every k_picture occupancy */
#define M2D_SHARE_UNITS_PER_CU 60

typedef struct m2d_share m2d_share_t;
/* the segment of device `key` (its PCI bus id) for this user (or group), created with `cap_units` if it does not
 * exist.  NULL with *why (optional) = M2D_SHARE_UNAVAILABLE when shared memory is unavailable here (the caller may
 * keep a process-local budget), M2D_SHARE_REFUSED when the file is not a valid segment of this version or its
 * leases are all held (reported on stderr: the caller must not decode with a private budget) */
#define M2D_SHARE_UNAVAILABLE 1
#define M2D_SHARE_REFUSED 2
m2d_share_t *m2d_share_open(const char *key, int cap_units, int *why);
/* 1: `units` reserved for this process; 0: they do not fit now (the leases of dead processes were reclaimed
 * first); -1: the segment is corrupted (reported).  total / procs (optional): the units in use and the
 * processes holding some, after the call */
int m2d_share_try(m2d_share_t *s, int units, int *total, int *procs);
void m2d_share_release(m2d_share_t *s, int units);
/* 1 when another process waits for units (a reservation of its that did not fit, within the last 100 ms) */
int m2d_share_others_waiting(m2d_share_t *s);
/* add `delta` to this process's live decode contexts; returns the device-wide count */
int m2d_share_contexts(m2d_share_t *s, int delta);
int m2d_share_state(m2d_share_t *s, int *cap, int *total, int *mine, int *procs, long *reclaimed);
int m2d_share_cap(const m2d_share_t *s);
void m2d_share_close(m2d_share_t *s);

#ifdef __cplusplus
}
#endif
#endif
