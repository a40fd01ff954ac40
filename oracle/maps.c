/*
 * ORACLE (test infrastructure only) -- see oracle.h.
 *
 * Restatement of bpftime's userspace maps as the helpers see them:
 *   ARRAY          runtime/src/bpf_map/userspace/array_map.cpp:19-81
 *   HASH (default) fix_size_hash_map_impl  fix_hash_map.cpp:16-84 over
 *                  bpftime_hash_map        runtime/src/bpf_map/bpftime_hash_map.hpp:12-205
 *                  (selected by map_handler.cpp:54-58, 785-798)
 *   PERCPU_ARRAY   per_cpu_array_map.cpp:17-145 (layout [idx][cpu][value])
 *   PERCPU_HASH    per_cpu_hash_map.cpp:20-216 (boost unordered_map in the
 *                  reference; here insertion-ordered, so get_next_key order
 *                  differs -> compared as key/value sets)
 *   flags check    map_common_def.hpp:83-94
 *   fd validity    bpftime_shm_internal.cpp:129-166, 457-466
 *   lddw helpers   bpftime_shm.cpp:637-676
 */
#include "oracle.h"
#include <errno.h>
#include <stdlib.h>
#include <string.h>

enum { T_HASH = 1, T_ARRAY = 2, T_PROG_ARRAY = 3, T_PERCPU_HASH = 5, T_PERCPU_ARRAY = 6, T_LRU_HASH = 9, T_LPM_TRIE = 11,
       T_RINGBUF = 27 };

struct orc_map {
	int used;
	uint32_t type, ksize, vsize, max_entries, flags;
	/* ARRAY / PERCPU_ARRAY */
	uint8_t *data;
	uint32_t ncpu;
	/* HASH: bpftime_hash_map layout [u32 used][key][value] per bucket */
	uint64_t nbuckets, count;
	/* PERCPU_HASH: keys[i], vals[i] (ncpu*vsize), insertion ordered */
	uint8_t *pkeys, *pvals;
	uint64_t pcount, pcap;
	/* key -> position + 1, open addressing; a lookup aid only (positions
	 * keep the insertion order the maps' iteration follows), rebuilt after
	 * an erase shifts the positions */
	uint32_t *pix;
	uint64_t pix_cap;
	int pix_valid;
	/* LPM_TRIE: node pool (lpm_trie_map.cpp keeps heap nodes; same tree) */
	struct lpm_node *nodes;
	int64_t nnodes, ncap, root;
	uint64_t lpm_entries;
	uint8_t *tl_value; /* the reference returns a thread-local copy */
	/* LRU_HASH (lru_var_hash_map.cpp): keys[i], vals[i], last-use stamps; the
	 * reference's recency list is the stamp order (head = largest stamp) */
	uint8_t *lkeys, *lvals;
	uint64_t *lstamp;
	uint64_t lcount, lclock;
	/* RINGBUF (ringbuf_map.cpp): consumer / producer positions, 2 x max_ent data */
	uint64_t rb_cons, rb_prod;
};
#define RB_PREFIX 8 /* zero bytes allocated in front of a ring's data */

struct lpm_node {
	uint32_t prefixlen;
	int intermediate;
	int64_t child[2];
	uint8_t *data; /* data_size prefix bytes, then value_size value bytes */
};

static struct orc_map g_maps[ORC_MAX_FDS];
static int g_ncpu = 1;
static int g_cpu = 0;
static __thread int g_errno;

int orc_last_errno(void)
{
	return g_errno;
}

void orc_set_ncpu(int ncpu)
{
	g_ncpu = ncpu > 0 ? ncpu : 1;
}

void orc_set_cpu(int cpu)
{
	g_cpu = cpu;
}

int orc_get_cpu(void)
{
	return g_cpu;
}

static void free_lpm(struct orc_map *m)
{
	for (int64_t i = 0; i < m->nnodes; i++)
		free(m->nodes[i].data);
	free(m->nodes);
	free(m->tl_value);
}

static void free_map(struct orc_map *m)
{
	if (m->type == T_LPM_TRIE)
		free_lpm(m);
	free(m->type == T_RINGBUF && m->data ? m->data - RB_PREFIX : m->data);
	free(m->pkeys);
	free(m->pix);
	free(m->pvals);
	free(m->lkeys);
	free(m->lvals);
	free(m->lstamp);
	memset(m, 0, sizeof(*m));
}

void orc_maps_reset(void)
{
	for (int fd = 0; fd < ORC_MAX_FDS; fd++)
		orc_prog_close(fd);
	for (int i = 0; i < ORC_MAX_FDS; i++)
		free_map(&g_maps[i]);
}

/* bpftime_hash_map.hpp:14-38 */
static int is_prime(uint64_t n)
{
	if (n <= 1)
		return 0;
	if (n <= 3)
		return 1;
	if (n % 2 == 0 || n % 3 == 0)
		return 0;
	for (uint64_t i = 5; i * i <= n; i += 6)
		if (n % i == 0 || n % (i + 2) == 0)
			return 0;
	return 1;
}

uint64_t orc_next_prime(uint64_t n)
{
	while (!is_prime(n))
		++n;
	return n;
}

/* bpftime_hash_map.hpp:40-47: h = h*31 + byte over size_t */
uint64_t orc_hash_bytes(const void *key, uint64_t n)
{
	uint64_t h = 0;
	for (uint64_t i = 0; i < n; i++)
		h = h * 31 + ((const uint8_t *)key)[i];
	return h;
}

static struct orc_map *get(int fd)
{
	if (fd < 0 || fd >= ORC_MAX_FDS || !g_maps[fd].used) {
		g_errno = ENOENT;
		return NULL;
	}
	return &g_maps[fd];
}

int orc_map_create(int fd, uint32_t type, uint32_t ksize, uint32_t vsize, uint32_t max_entries,
		   uint32_t flags)
{
	if (fd < 0) {
		for (fd = 3; fd < ORC_MAX_FDS && g_maps[fd].used; fd++)
			;
	}
	if (fd >= ORC_MAX_FDS || g_maps[fd].used)
		return -1;
	struct orc_map *m = &g_maps[fd];
	memset(m, 0, sizeof(*m));
	m->type = type;
	m->ksize = ksize;
	m->vsize = vsize;
	m->max_entries = max_entries;
	m->flags = flags;
	switch (type) {
	case T_ARRAY:
		m->data = calloc((size_t)vsize * max_entries + 1, 1);
		break;
	case T_PERCPU_ARRAY:
		m->ncpu = (uint32_t)g_ncpu;
		m->data = calloc((size_t)vsize * max_entries * m->ncpu + 1, 1);
		break;
	case T_HASH:
		m->nbuckets = orc_next_prime(max_entries);
		m->data = calloc((size_t)m->nbuckets * (4 + ksize + vsize) + 1, 1);
		break;
	case T_PERCPU_HASH:
		m->ncpu = (uint32_t)g_ncpu;
		break;
	case T_LRU_HASH: /* lru_var_hash_map.cpp:13-25 (max_entries 0 would evict from an empty list) */
		if (ksize == 0 || vsize == 0 || max_entries == 0) {
			g_errno = EINVAL;
			return -1;
		}
		m->lkeys = malloc((size_t)max_entries * ksize);
		m->lvals = malloc((size_t)max_entries * vsize);
		m->lstamp = malloc((size_t)max_entries * 8);
		break;
	case T_PROG_ARRAY: /* prog_array.cpp:101-110: every slot INVALID_ENTRY (-1) */
		if (ksize != 4 || vsize != 4) {
			g_errno = EINVAL;
			return -1;
		}
		m->data = malloc((size_t)max_entries * 4 + 1);
		memset(m->data, 0xff, (size_t)max_entries * 4);
		break;
	case T_RINGBUF: /* ringbuf_map.cpp ringbuf::ringbuf: data = 2 x max_ent bytes */
		if (max_entries == 0 || (max_entries & (max_entries - 1))) {
			g_errno = EINVAL;
			return -1;
		}
		/* behind data: the zeroed tail of the reference's producer page
		 * (raw_buffer[2 * page - RB_PREFIX ..]), which bpf_ringbuf_submit's
		 * ptr[-1] reads as the fd of a record whose data wrapped to data[0] */
		m->data = calloc((size_t)max_entries * 2 + RB_PREFIX, 1);
		if (m->data)
			m->data += RB_PREFIX;
		break;
	case T_LPM_TRIE: /* lpm_trie_map.cpp:43-81: key = u32 prefixlen + 1..256 data bytes */
		if (ksize < 5 || ksize > 260 || vsize == 0 || max_entries == 0) {
			g_errno = EINVAL;
			return -1;
		}
		m->root = -1;
		m->tl_value = calloc(vsize, 1);
		break;
	default:
		return -1;
	}
	m->used = 1;
	return fd;
}

/* map_common_def.hpp:83-94 */
static int check_update_flags(uint64_t flags)
{
	uint64_t b = flags & 0xffffffffULL;
	if (b != 0 && b != 1 && b != 2) {
		g_errno = EINVAL;
		return 0;
	}
	return 1;
}

/* ---- fix-size hash (bpftime_hash_map.hpp) ---- */
static inline uint8_t *slot(struct orc_map *m, uint64_t i)
{
	return m->data + i * (4 + m->ksize + m->vsize);
}

static void *hash_lookup(struct orc_map *m, const void *key)
{
	uint64_t idx = orc_hash_bytes(key, m->ksize) % m->nbuckets, start = idx;
	do {
		uint8_t *s = slot(m, idx);
		if (*(uint32_t *)s == 0)
			return NULL;
		if (memcmp(s + 4, key, m->ksize) == 0)
			return s + 4 + m->ksize;
		idx = (idx + 1) % m->nbuckets;
	} while (idx != start);
	return NULL;
}

static int hash_update(struct orc_map *m, const void *key, const void *val)
{
	uint64_t idx = orc_hash_bytes(key, m->ksize) % m->nbuckets, start = idx;
	do {
		uint8_t *s = slot(m, idx);
		if (*(uint32_t *)s == 0) {
			if (m->count >= m->max_entries)
				return 0; /* full: reject (:153-156) */
			memcpy(s + 4, key, m->ksize);
			memcpy(s + 4 + m->ksize, val, m->vsize);
			*(uint32_t *)s = 1;
			m->count++;
			return 1;
		} else if (memcmp(s + 4, key, m->ksize) == 0) {
			memcpy(s + 4 + m->ksize, val, m->vsize);
			return 1;
		}
		idx = (idx + 1) % m->nbuckets;
	} while (idx != start);
	return 0;
}

static int hash_delete(struct orc_map *m, const void *key)
{
	uint64_t idx = orc_hash_bytes(key, m->ksize) % m->nbuckets, start = idx;
	do {
		uint8_t *s = slot(m, idx);
		if (*(uint32_t *)s == 0)
			return 0;
		if (memcmp(s + 4, key, m->ksize) == 0) {
			*(uint32_t *)s = 0; /* no tombstone (:182-199) */
			m->count--;
			return 1;
		}
		idx = (idx + 1) % m->nbuckets;
	} while (idx != start);
	return 0;
}

/* ---- per-cpu hash (per_cpu_hash_map.cpp) ---- */
static uint64_t pix_hash(const void *key, uint32_t n) /* FNV-1a */
{
	uint64_t h = 1469598103934665603ull;
	for (uint32_t i = 0; i < n; i++)
		h = (h ^ ((const uint8_t *)key)[i]) * 1099511628211ull;
	return h ^ (h >> 29);
}

static void pix_put(struct orc_map *m, uint64_t i)
{
	uint64_t p = pix_hash(m->pkeys + i * m->ksize, m->ksize) & (m->pix_cap - 1);
	while (m->pix[p])
		p = (p + 1) & (m->pix_cap - 1);
	m->pix[p] = (uint32_t)i + 1;
}

static void pix_rebuild(struct orc_map *m)
{
	uint64_t cap = 64;
	while (cap < 4 * (m->pcount + 1))
		cap *= 2;
	free(m->pix);
	m->pix = calloc(cap, 4);
	m->pix_cap = cap;
	for (uint64_t i = 0; i < m->pcount; i++)
		pix_put(m, i);
	m->pix_valid = 1;
}

static int64_t phash_find(struct orc_map *m, const void *key)
{
	if (!m->pix_valid || m->pix_cap < 2 * (m->pcount + 1))
		pix_rebuild(m);
	uint64_t p = pix_hash(key, m->ksize) & (m->pix_cap - 1);
	for (; m->pix[p]; p = (p + 1) & (m->pix_cap - 1))
		if (memcmp(m->pkeys + (uint64_t)(m->pix[p] - 1) * m->ksize, key, m->ksize) == 0)
			return (int64_t)m->pix[p] - 1;
	return -1;
}

static uint64_t phash_insert(struct orc_map *m, const void *key)
{
	if (m->pcount == m->pcap) {
		m->pcap = m->pcap ? m->pcap * 2 : 16;
		m->pkeys = realloc(m->pkeys, m->pcap * m->ksize);
		m->pvals = realloc(m->pvals, m->pcap * (size_t)m->ncpu * m->vsize);
	}
	uint64_t i = m->pcount++;
	memcpy(m->pkeys + i * m->ksize, key, m->ksize);
	memset(m->pvals + i * (size_t)m->ncpu * m->vsize, 0, (size_t)m->ncpu * m->vsize);
	if (m->pix_valid && m->pix_cap >= 2 * (m->pcount + 1))
		pix_put(m, i);
	else
		m->pix_valid = 0;
	return i;
}

static void phash_erase(struct orc_map *m, uint64_t i)
{
	size_t vs = (size_t)m->ncpu * m->vsize;
	memmove(m->pkeys + i * m->ksize, m->pkeys + (i + 1) * m->ksize, (m->pcount - i - 1) * m->ksize);
	memmove(m->pvals + i * vs, m->pvals + (i + 1) * vs, (m->pcount - i - 1) * vs);
	m->pcount--;
	m->pix_valid = 0;
}

/* ---- LRU hash (runtime/src/bpf_map/userspace/lru_var_hash_map.cpp) ----
 * The reference keeps a boost unordered_map plus a doubly linked recency list
 * (head = most recent).  Here each element carries the clock value of its
 * last use: move_to_head (:137-161) = a new, largest stamp, the list tail =
 * the smallest stamp, evict_entry (:189-221) = removal.  Same observable
 * contents and eviction victims. */
static int64_t lru_find(struct orc_map *m, const void *key)
{
	for (uint64_t i = 0; i < m->lcount; i++)
		if (memcmp(m->lkeys + i * m->ksize, key, m->ksize) == 0)
			return (int64_t)i;
	return -1;
}

static void lru_erase(struct orc_map *m, uint64_t i)
{
	uint64_t last = m->lcount - 1;
	if (i != last) {
		memcpy(m->lkeys + i * m->ksize, m->lkeys + last * m->ksize, m->ksize);
		memcpy(m->lvals + i * m->vsize, m->lvals + last * m->vsize, m->vsize);
		m->lstamp[i] = m->lstamp[last];
	}
	m->lcount--;
}

static void *lru_lookup(struct orc_map *m, const void *key) /* :27-41 */
{
	int64_t i = key ? lru_find(m, key) : -1;
	if (i < 0) {
		g_errno = ENOENT;
		return NULL;
	}
	m->lstamp[i] = ++m->lclock; /* move_to_head */
	return m->lvals + (size_t)i * m->vsize;
}

static long lru_update(struct orc_map *m, const void *key, const void *value, uint64_t flags) /* :43-90 */
{
	if (flags != 0 && flags != 1 && flags != 2) { /* is_good_update_flag (:8-11): exact values */
		g_errno = EINVAL;
		return -1;
	}
	int64_t i = lru_find(m, key);
	if (flags == 1 /*BPF_NOEXIST*/ && i >= 0) {
		g_errno = EEXIST;
		return -1;
	}
	if (flags == 2 /*BPF_EXIST*/ && i < 0) {
		g_errno = ENOENT;
		return -1;
	}
	if (i < 0 && m->lcount == m->max_entries) { /* evict the list tail */
		uint64_t t = 0;
		for (uint64_t j = 1; j < m->lcount; j++)
			if (m->lstamp[j] < m->lstamp[t])
				t = j;
		lru_erase(m, t);
	}
	if (i < 0) { /* insert_new_entry (:163-187): at the head */
		i = (int64_t)m->lcount++;
		memcpy(m->lkeys + (size_t)i * m->ksize, key, m->ksize);
	}
	memcpy(m->lvals + (size_t)i * m->vsize, value, m->vsize);
	m->lstamp[i] = ++m->lclock;
	return 0;
}

static long lru_delete(struct orc_map *m, const void *key) /* :92-103 */
{
	int64_t i = lru_find(m, key);
	if (i < 0) {
		g_errno = ENOENT;
		return -1;
	}
	lru_erase(m, (uint64_t)i);
	return 0;
}

/* :105-135.  The reference walks its unordered_map's order, which is not
 * part of its contract (its tests compare visited sets); this walks element
 * slots.  A key that is not present restarts at the first key. */
static int lru_next_key(struct orc_map *m, const void *key, void *next)
{
	int64_t i = key ? lru_find(m, key) : -1;
	uint64_t nx = i < 0 ? 0 : (uint64_t)i + 1;
	if (nx >= m->lcount) {
		g_errno = ENOENT;
		return -1;
	}
	memcpy(next, m->lkeys + nx * m->ksize, m->ksize);
	return 0;
}

/* ---- helper-side ops (bpf_map_handler::map_*_elem, from_syscall=false) ---- */


/* ---- ring buffer (runtime/src/bpf_map/userspace/ringbuf_map.cpp) ---- */
#define RB_BUSY 0x80000000u
#define RB_DISCARD 0x40000000u
#define RB_HDR 8

void *orc_ringbuf_reserve(int fd, uint64_t size) /* ringbuf::reserve */
{
	struct orc_map *m = get(fd);
	if (!m || m->type != T_RINGBUF)
		return NULL;
	if (size & (RB_BUSY | RB_DISCARD)) {
		g_errno = E2BIG;
		return NULL;
	}
	uint64_t mask = m->max_entries - 1;
	uint64_t avail = m->max_entries - (m->rb_prod - m->rb_cons);
	uint64_t total = (size + RB_HDR + 7) / 8 * 8;
	if (total > m->max_entries) {
		g_errno = E2BIG;
		return NULL;
	}
	if (avail < total) {
		g_errno = ENOSPC;
		return NULL;
	}
	uint8_t *hdr = m->data + (m->rb_prod & mask);
	*(uint32_t *)hdr = (uint32_t)size | RB_BUSY;
	*(int32_t *)(hdr + 4) = fd;
	uint8_t *ptr = m->data + ((m->rb_prod + RB_HDR) & mask);
	m->rb_prod += total;
	return ptr;
}

/* bpftime_ringbuf_submit(fd, sample, discard) (bpftime_shm.cpp:401-411) ->
 * ringbuf::submit (ringbuf_map.cpp:297-309) */
void orc_ringbuf_submit_fd(int fd, const void *sample, int discard)
{
	struct orc_map *m = get(fd);
	if (!m || m->type != T_RINGBUF)
		return;
	uint64_t mask = m->max_entries - 1;
	uint64_t off = (mask + 1 + (uint64_t)((const uint8_t *)sample - m->data) - RB_HDR) & mask;
	uint32_t *len = (uint32_t *)(m->data + off);
	uint32_t v = *len & ~RB_BUSY;
	if (discard)
		v |= RB_DISCARD;
	*len = v;
}

/* ringbuf::fetch_data: committed, non-discarded records in order, each
 * written to out as [u32 len][len bytes]; returns the record count */
int64_t orc_ringbuf_fetch(int fd, uint8_t *out, uint64_t cap, uint64_t *used)
{
	struct orc_map *m = get(fd);
	*used = 0;
	if (!m || m->type != T_RINGBUF)
		return -1;
	uint64_t mask = m->max_entries - 1;
	int64_t cnt = 0;
	while (m->rb_cons < m->rb_prod) {
		uint32_t len = *(uint32_t *)(m->data + (m->rb_cons & mask));
		if (len & RB_BUSY)
			break;
		uint32_t n = len & ~(RB_BUSY | RB_DISCARD);
		if (!(len & RB_DISCARD)) {
			if (*used + 4 + n > cap)
				break;
			memcpy(out + *used, &n, 4);
			memcpy(out + *used + 4, m->data + (m->rb_cons & mask) + RB_HDR, n);
			*used += 4 + n;
			cnt++;
		}
		m->rb_cons += ((uint64_t)n + RB_HDR + 7) / 8 * 8;
	}
	return cnt;
}

/* ---- LPM trie (runtime/src/bpf_map/userspace/lpm_trie_map.cpp) ---- */
static uint32_t lpm_dsz(const struct orc_map *m)
{
	return m->ksize - 4;
}

static int lpm_bit(const struct orc_map *m, const uint8_t *d, size_t i) /* :88-98 */
{
	if (i >= (size_t)lpm_dsz(m) * 8)
		return 0;
	return (d[i / 8] >> (7 - (i % 8))) & 1;
}

static size_t lpm_match(const struct orc_map *m, const struct lpm_node *n, const uint8_t *key) /* :101-113 */
{
	uint32_t kp = *(const uint32_t *)key;
	uint32_t lim = n->prefixlen < kp ? n->prefixlen : kp;
	size_t i = 0;
	for (; i < lim; i++)
		if (lpm_bit(m, n->data, i) != lpm_bit(m, key + 4, i))
			break;
	return i;
}

static int64_t lpm_new(struct orc_map *m, const uint8_t *key, uint32_t plen, const void *value, int inter)
{
	if (m->nnodes == m->ncap) {
		m->ncap = m->ncap ? 2 * m->ncap : 16;
		m->nodes = realloc(m->nodes, (size_t)m->ncap * sizeof(struct lpm_node));
	}
	struct lpm_node *n = &m->nodes[m->nnodes];
	n->prefixlen = plen;
	n->intermediate = inter;
	n->child[0] = n->child[1] = -1;
	n->data = calloc(lpm_dsz(m) + m->vsize, 1);
	memcpy(n->data, key + 4, lpm_dsz(m));
	if (!inter && value)
		memcpy(n->data + lpm_dsz(m), value, m->vsize);
	return m->nnodes++;
}

static void *lpm_lookup(struct orc_map *m, const uint8_t *key) /* :192-264 */
{
	const uint32_t maxp = lpm_dsz(m) * 8, kp = *(const uint32_t *)key;
	if (kp > maxp) {
		g_errno = EINVAL;
		return NULL;
	}
	int64_t node = m->root, found = -1;
	while (node >= 0) {
		struct lpm_node *n = &m->nodes[node];
		size_t ml = lpm_match(m, n, key);
		if (ml == maxp) {
			found = node;
			break;
		}
		if (ml < n->prefixlen)
			break;
		if (!n->intermediate)
			found = node;
		if (ml < kp)
			node = n->child[lpm_bit(m, key + 4, n->prefixlen)];
		else
			break;
	}
	if (found < 0 || m->nodes[found].intermediate) {
		g_errno = ENOENT;
		return NULL;
	}
	memcpy(m->tl_value, m->nodes[found].data + lpm_dsz(m), m->vsize);
	return m->tl_value;
}

static long lpm_update(struct orc_map *m, const uint8_t *key, const void *value, uint64_t flags) /* :266-488 */
{
	if (flags != 0 && flags != 1 && flags != 2) {
		g_errno = EINVAL;
		return -1;
	}
	const uint32_t maxp = lpm_dsz(m) * 8, kp = *(const uint32_t *)key;
	if (kp > maxp) {
		g_errno = EINVAL;
		return -1;
	}
#define LPM_NEED_ROOM()                                   \
	do {                                              \
		if (flags == 2) {                         \
			g_errno = ENOENT;                 \
			return -1;                        \
		}                                         \
		if (m->lpm_entries >= m->max_entries) {   \
			g_errno = ENOSPC;                 \
			return -1;                        \
		}                                         \
	} while (0)
	if (m->root < 0) {
		LPM_NEED_ROOM();
		m->root = lpm_new(m, key, kp, value, 0);
		m->lpm_entries++;
		return 0;
	}
	int64_t *slotp = &m->root, node = -1;
	size_t ml = 0;
	/* walk (slot pointers are indices into nodes[]: re-derived after lpm_new) */
	int64_t parent = -2;
	int pbit = 0;
	while (*slotp >= 0) {
		node = *slotp;
		struct lpm_node *n = &m->nodes[node];
		ml = lpm_match(m, n, key);
		if (n->prefixlen != ml || n->prefixlen == kp || n->prefixlen == maxp)
			break;
		pbit = lpm_bit(m, key + 4, n->prefixlen);
		parent = node;
		slotp = &n->child[pbit];
	}
#define SLOT_SET(v)                                       \
	do {                                              \
		int64_t v_ = (v);                         \
		if (parent == -2)                         \
			m->root = v_;                     \
		else                                      \
			m->nodes[parent].child[pbit] = v_; \
	} while (0)
	const int64_t cur = *slotp;
	if (cur >= 0 && m->nodes[cur].prefixlen == kp) { /* case 1 */
		struct lpm_node *n = &m->nodes[cur];
		if (lpm_match(m, n, key) == kp) {
			int real = !n->intermediate;
			if (flags == 1) {
				g_errno = EEXIST;
				return -1;
			}
			if (flags == 2 && !real) {
				g_errno = ENOENT;
				return -1;
			}
			if (!real) {
				if (m->lpm_entries >= m->max_entries) {
					g_errno = ENOSPC;
					return -1;
				}
				n->intermediate = 0;
				m->lpm_entries++;
			}
			memcpy(n->data + lpm_dsz(m), value, m->vsize);
			return 0;
		}
		LPM_NEED_ROOM();
		int64_t nn = lpm_new(m, key, kp, value, 0);
		int64_t im = lpm_new(m, key, (uint32_t)ml, NULL, 1);
		if (lpm_bit(m, key + 4, ml)) {
			m->nodes[im].child[0] = cur;
			m->nodes[im].child[1] = nn;
		} else {
			m->nodes[im].child[0] = nn;
			m->nodes[im].child[1] = cur;
		}
		SLOT_SET(im);
		m->lpm_entries++;
		return 0;
	}
	if (cur < 0) { /* case 2 */
		LPM_NEED_ROOM();
		int64_t nn = lpm_new(m, key, kp, value, 0);
		SLOT_SET(nn);
		m->lpm_entries++;
		return 0;
	}
	if (ml == kp) { /* case 3: the new prefix becomes cur's parent */
		LPM_NEED_ROOM();
		int64_t nn = lpm_new(m, key, kp, value, 0);
		int nb = lpm_bit(m, m->nodes[cur].data, ml);
		m->nodes[nn].child[nb] = cur;
		SLOT_SET(nn);
		m->lpm_entries++;
		return 0;
	}
	LPM_NEED_ROOM(); /* case 4: intermediate node at the split */
	int64_t nn = lpm_new(m, key, kp, value, 0);
	int64_t im = lpm_new(m, key, (uint32_t)ml, NULL, 1);
	if (lpm_bit(m, key + 4, ml)) {
		m->nodes[im].child[0] = cur;
		m->nodes[im].child[1] = nn;
	} else {
		m->nodes[im].child[0] = nn;
		m->nodes[im].child[1] = cur;
	}
	SLOT_SET(im);
	m->lpm_entries++;
	return 0;
#undef SLOT_SET
#undef LPM_NEED_ROOM
}

static long lpm_delete(struct orc_map *m, const uint8_t *key) /* :490-541: logical deletion */
{
	const uint32_t maxp = lpm_dsz(m) * 8, kp = *(const uint32_t *)key;
	if (kp > maxp) {
		g_errno = EINVAL;
		return -1;
	}
	int64_t node = m->root, last = -1;
	while (node >= 0) {
		struct lpm_node *n = &m->nodes[node];
		last = node;
		size_t ml = lpm_match(m, n, key);
		if (n->prefixlen != ml || n->prefixlen == kp)
			break;
		node = n->child[lpm_bit(m, key + 4, n->prefixlen)];
		last = node;
	}
	if (last < 0 || m->nodes[last].prefixlen != kp || lpm_match(m, &m->nodes[last], key) != kp ||
	    m->nodes[last].intermediate) {
		g_errno = ENOENT;
		return -1;
	}
	m->nodes[last].intermediate = 1;
	memset(m->nodes[last].data + lpm_dsz(m), 0, m->vsize);
	if (m->lpm_entries > 0)
		m->lpm_entries--;
	return 0;
}

static int lpm_next_key(struct orc_map *m, const void *key, uint8_t *next) /* :543-590 */
{
	if (m->root < 0 || key) { /* only the first key is implemented by the reference */
		g_errno = ENOENT;
		return -1;
	}
	int64_t node = m->root;
	while (node >= 0) {
		struct lpm_node *n = &m->nodes[node];
		if (!n->intermediate) {
			*(uint32_t *)next = n->prefixlen;
			memcpy(next + 4, n->data, lpm_dsz(m));
			return 0;
		}
		node = n->child[0] >= 0 ? n->child[0] : n->child[1];
	}
	g_errno = ENOENT;
	return -1;
}

/* ---- PROG_ARRAY (prog_array.cpp); slots hold bpftime prog fds ---- */
static __thread int32_t tl_prog_fd;

int orc_map_is_prog_array(int fd)
{
	struct orc_map *m = get(fd);
	return m && m->type == T_PROG_ARRAY;
}

static void *parr_lookup(struct orc_map *m, const void *key) /* prog_array.cpp:113-143 */
{
	int32_t k = *(const int32_t *)key;
	if (k < 0 || (uint32_t)k >= m->max_entries) {
		g_errno = EINVAL;
		return NULL;
	}
	int32_t v = ((const int32_t *)m->data)[k];
	if (v < 0 || !orc_is_prog_fd(v)) {
		g_errno = ENOENT;
		return NULL;
	}
	tl_prog_fd = v;
	return &tl_prog_fd;
}

static long parr_update(struct orc_map *m, const void *key, const void *value) /* :146-176 */
{
	int32_t k = *(const int32_t *)key, v = *(const int32_t *)value;
	if (k < 0 || (uint32_t)k >= m->max_entries) {
		g_errno = EINVAL;
		return -1;
	}
	if (!orc_is_prog_fd(v)) { /* would be asked of the kernel: no such fd */
		g_errno = EBADF;
		return -1;
	}
	((int32_t *)m->data)[k] = v;
	return 0;
}

static long parr_delete(struct orc_map *m, const void *key) /* :180-189 */
{
	int32_t k = *(const int32_t *)key;
	if (k < 0 || (uint32_t)k >= m->max_entries) {
		g_errno = EINVAL;
		return -1;
	}
	((int32_t *)m->data)[k] = -1;
	return 0;
}

static int parr_next_key(struct orc_map *m, const void *key, void *next) /* :191-211 */
{
	if (!key) {
		*(int32_t *)next = 0;
		return 0;
	}
	int32_t k = *(const int32_t *)key;
	if ((size_t)(k + 1) == m->max_entries) {
		g_errno = ENOENT;
		return -1;
	}
	if (k < 0 || (uint32_t)k >= m->max_entries) {
		g_errno = EINVAL;
		return -1;
	}
	*(int32_t *)next = k + 1;
	return 0;
}

void *orc_map_lookup(int fd, const void *key)
{
	struct orc_map *m = get(fd);
	if (!m)
		return NULL;
	switch (m->type) {
	case T_PROG_ARRAY:
		return parr_lookup(m, key);
	case T_ARRAY: { /* array_map.cpp:27-35 */
		uint32_t k = *(const uint32_t *)key;
		if (k >= m->max_entries) {
			g_errno = ENOENT;
			return NULL;
		}
		return m->data + (size_t)k * m->vsize;
	}
	case T_PERCPU_ARRAY: { /* per_cpu_array_map.cpp:34-48 */
		if (!key) {
			g_errno = ENOENT;
			return NULL;
		}
		uint32_t k = *(const uint32_t *)key;
		if (k >= m->max_entries) {
			g_errno = ENOENT;
			return NULL;
		}
		return m->data + ((size_t)k * m->ncpu + (size_t)g_cpu) * m->vsize;
	}
	case T_HASH:
		return hash_lookup(m, key);
	case T_LRU_HASH:
		return lru_lookup(m, key);
	case T_LPM_TRIE:
		return key ? lpm_lookup(m, key) : NULL;
	case T_RINGBUF:
		g_errno = ENOTSUP;
		return NULL;
	case T_PERCPU_HASH: { /* per_cpu_hash_map.cpp:48-64 */
		if (!key) {
			g_errno = ENOENT;
			return NULL;
		}
		int64_t i = phash_find(m, key);
		if (i < 0) {
			g_errno = ENOENT;
			return NULL;
		}
		return m->pvals + ((size_t)i * m->ncpu + (size_t)g_cpu) * m->vsize;
	}
	}
	return NULL;
}

long orc_map_update(int fd, const void *key, const void *value, uint64_t flags)
{
	struct orc_map *m = get(fd);
	if (!m)
		return -1;
	switch (m->type) {
	case T_PROG_ARRAY:
		return parr_update(m, key, value);
	case T_ARRAY: /* array_map.cpp:37-56 */
	case T_PERCPU_ARRAY: { /* per_cpu_array_map.cpp:50-73 */
		if (!check_update_flags(flags))
			return -1;
		uint32_t k = *(const uint32_t *)key;
		if (k < m->max_entries && flags == 1 /*BPF_NOEXIST*/) {
			g_errno = EEXIST;
			return -1;
		}
		if (k >= m->max_entries) {
			g_errno = E2BIG;
			return -1;
		}
		uint8_t *dst = m->type == T_ARRAY ? m->data + (size_t)k * m->vsize
						  : m->data + ((size_t)k * m->ncpu + (size_t)g_cpu) * m->vsize;
		memcpy(dst, value, m->vsize);
		return 0;
	}
	case T_LPM_TRIE:
		return lpm_update(m, key, value, flags);
	case T_LRU_HASH:
		return lru_update(m, key, value, flags);
	case T_HASH: /* fix_hash_map.cpp:34-39: flags ignored, always 0 */
		hash_update(m, key, value);
		return 0;
	case T_PERCPU_HASH: { /* per_cpu_hash_map.cpp:66-94: no max-entries check */
		if (!check_update_flags(flags))
			return -1;
		int64_t i = phash_find(m, key);
		if (i < 0)
			i = (int64_t)phash_insert(m, key);
		memcpy(m->pvals + ((size_t)i * m->ncpu + (size_t)g_cpu) * m->vsize, value, m->vsize);
		return 0;
	}
	}
	return -1;
}

long orc_map_delete(int fd, const void *key)
{
	struct orc_map *m = get(fd);
	if (!m)
		return -1;
	switch (m->type) {
	case T_PROG_ARRAY:
		return parr_delete(m, key);
	case T_ARRAY:
	case T_PERCPU_ARRAY: /* array_map.cpp:58-64 */
		g_errno = EINVAL;
		return -1;
	case T_HASH: /* fix_hash_map.cpp:41-45 */
		hash_delete(m, key);
		return 0;
	case T_LPM_TRIE:
		return lpm_delete(m, key);
	case T_LRU_HASH:
		return lru_delete(m, key);
	case T_PERCPU_HASH: { /* per_cpu_hash_map.cpp:96-107: zeroes [0, cpu*vsize) */
		int64_t i = phash_find(m, key);
		if (i >= 0)
			memset(m->pvals + (size_t)i * m->ncpu * m->vsize, 0, (size_t)g_cpu * m->vsize);
		return 0;
	}
	}
	return -1;
}

/* ---- syscall-side ops (from_syscall=true) ---- */
void *orc_map_lookup_user(int fd, const void *key)
{
	struct orc_map *m = get(fd);
	if (!m)
		return NULL;
	if (m->type == T_PERCPU_ARRAY) { /* per_cpu_array_map.cpp:97-108 */
		uint32_t k = *(const uint32_t *)key;
		if (k >= m->max_entries) {
			g_errno = ENOENT;
			return NULL;
		}
		return m->data + (size_t)k * m->ncpu * m->vsize;
	}
	if (m->type == T_PERCPU_HASH) { /* per_cpu_hash_map.cpp:141-155 */
		int64_t i = phash_find(m, key);
		if (i < 0) {
			g_errno = ENOENT;
			return NULL;
		}
		return m->pvals + (size_t)i * m->ncpu * m->vsize;
	}
	return orc_map_lookup(fd, key);
}

long orc_map_update_user(int fd, const void *key, const void *value, uint64_t flags)
{
	struct orc_map *m = get(fd);
	if (!m)
		return -1;
	if (m->type == T_PERCPU_ARRAY) { /* per_cpu_array_map.cpp:110-131 */
		if (!check_update_flags(flags))
			return -1;
		uint32_t k = *(const uint32_t *)key;
		if (k < m->max_entries && flags == 1) {
			g_errno = EEXIST;
			return -1;
		}
		if (k >= m->max_entries) {
			g_errno = E2BIG;
			return -1;
		}
		memcpy(m->data + (size_t)k * m->ncpu * m->vsize, value, (size_t)m->ncpu * m->vsize);
		return 0;
	}
	if (m->type == T_PERCPU_HASH) { /* per_cpu_hash_map.cpp:157-183 */
		if (!check_update_flags(flags))
			return -1;
		int64_t i = phash_find(m, key);
		if (flags == 1 && i >= 0) {
			g_errno = EEXIST;
			return -1;
		}
		if (flags == 2 && i < 0) {
			g_errno = ENOENT;
			return -1;
		}
		if (i < 0 && m->pcount == m->max_entries) {
			g_errno = E2BIG;
			return -1;
		}
		if (i < 0)
			i = (int64_t)phash_insert(m, key);
		memcpy(m->pvals + (size_t)i * m->ncpu * m->vsize, value, (size_t)m->ncpu * m->vsize);
		return 0;
	}
	return orc_map_update(fd, key, value, flags);
}

long orc_map_delete_user(int fd, const void *key)
{
	struct orc_map *m = get(fd);
	if (!m)
		return -1;
	if (m->type == T_PERCPU_HASH) { /* per_cpu_hash_map.cpp:184-195 */
		int64_t i = phash_find(m, key);
		if (i < 0) {
			g_errno = ENOENT;
			return -1;
		}
		phash_erase(m, (uint64_t)i);
		return 0;
	}
	return orc_map_delete(fd, key);
}

int orc_map_get_next_key(int fd, const void *key, void *next_key)
{
	struct orc_map *m = get(fd);
	if (!m)
		return -1;
	switch (m->type) {
	case T_PROG_ARRAY:
		return parr_next_key(m, key, next_key);
	case T_ARRAY:
	case T_PERCPU_ARRAY: /* array_map.cpp:66-81 */
		if (!key || *(const uint32_t *)key >= m->max_entries) {
			*(uint32_t *)next_key = 0;
			return 0;
		}
		if (*(const uint32_t *)key == m->max_entries - 1) {
			g_errno = ENOENT;
			return -1;
		}
		*(uint32_t *)next_key = *(const uint32_t *)key + 1;
		return 0;
	case T_HASH: { /* fix_hash_map.cpp:47-84: bucket index order */
		uint64_t from = 0;
		if (key) {
			uint8_t *v = hash_lookup(m, key);
			if (v)
				from = (uint64_t)(v - m->data) / (4 + m->ksize + m->vsize) + 1;
		}
		for (uint64_t i = from; i < m->nbuckets; i++) {
			uint8_t *s = slot(m, i);
			if (*(uint32_t *)s) {
				memcpy(next_key, s + 4, m->ksize);
				return 0;
			}
		}
		g_errno = ENOENT;
		return -1;
	}
	case T_LPM_TRIE:
		return lpm_next_key(m, key, next_key);
	case T_LRU_HASH:
		return lru_next_key(m, key, next_key);
	case T_PERCPU_HASH: {
		int64_t i = key ? phash_find(m, key) : -1;
		uint64_t nx = i < 0 ? 0 : (uint64_t)i + 1;
		if (nx >= m->pcount) {
			g_errno = ENOENT;
			return -1;
		}
		memcpy(next_key, m->pkeys + nx * m->ksize, m->ksize);
		return 0;
	}
	}
	return -1;
}

uint32_t orc_map_value_size_user(int fd)
{
	struct orc_map *m = get(fd);
	if (!m)
		return 0;
	if (m->type == T_PERCPU_ARRAY || m->type == T_PERCPU_HASH)
		return m->vsize * m->ncpu; /* map_handler.cpp:69-84 */
	return m->vsize;
}

void *orc_map_raw(int fd, size_t *bytes)
{
	struct orc_map *m = get(fd);
	if (!m)
		return NULL;
	switch (m->type) {
	case T_ARRAY:
		*bytes = (size_t)m->vsize * m->max_entries;
		return m->data;
	case T_PERCPU_ARRAY:
		*bytes = (size_t)m->vsize * m->max_entries * m->ncpu;
		return m->data;
	case T_HASH:
		*bytes = (size_t)m->nbuckets * (4 + m->ksize + m->vsize);
		return m->data;
	case T_PERCPU_HASH:
		*bytes = (size_t)m->pcount * m->ncpu * m->vsize;
		return m->pvals;
	}
	return NULL;
}

uint64_t orc_map_buckets(int fd)
{
	struct orc_map *m = get(fd);
	return m ? m->nbuckets : 0;
}

uint64_t orc_map_count(int fd)
{
	struct orc_map *m = get(fd);
	if (!m)
		return 0;
	return m->type == T_PERCPU_HASH ? m->pcount
	       : m->type == T_LPM_TRIE	 ? m->lpm_entries
	       : m->type == T_LRU_HASH	 ? m->lcount
					 : m->count;
}

/* bpftime_shm.cpp:637-652: the map "pointer" is the fd itself */
uint64_t orc_map_ptr_by_fd(uint32_t fd)
{
	if (!get((int)fd)) {
		g_errno = ENOENT;
		return ~0ULL;
	}
	return fd;
}

/* bpftime_shm.cpp:654-676: address of the value at get_next_key(NULL) */
uint64_t orc_map_val(uint64_t map_ptr)
{
	int fd = (int)map_ptr;
	struct orc_map *m = get(fd);
	if (!m) {
		g_errno = ENOENT;
		return 0;
	}
	uint8_t key[256] = {0};
	if (orc_map_get_next_key(fd, NULL, key) < 0) {
		g_errno = ENOENT;
		return 0;
	}
	return (uint64_t)(uintptr_t)orc_map_lookup(fd, key);
}
