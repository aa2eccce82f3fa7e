/*
 * errutil.c -- MPICH's error-code / error-stack interface for a standalone
 * build of this library.
 *
 * MPI_Reduce_local reports a failure the reference's way
 * (reduce_local.c:208-217):
 *     mpi_errno = MPIR_Err_create_code(mpi_errno, MPIR_ERR_RECOVERABLE, FCNAME, __LINE__,
 *                                      MPI_ERR_OTHER, "**mpi_reduce_local",
 *                                      "**mpi_reduce_local %p %p %d %D %O", ...);
 *     mpi_errno = MPIR_Err_return_comm(NULL, FCNAME, mpi_errno);
 * Every definition here is WEAK: when the host sources are compiled into
 * libmpi (Option 1) libmpi's own MPIR_Err_create_code
 * (errutil.c:848), MPIR_Err_return_comm (errutil.c:238), MPI_Error_class and
 * MPI_Error_string take over, and the codes, the error ring and the
 * communicator error handlers are MPICH's.
 *
 * Standalone, the codes follow MPICH's layout (src/mpi/errhan/errcodes.h:47-61):
 * class in bits 0-6, fatal bit 7, error-ring index in bits 19-25 and a ring
 * sequence number in bits 26-29, so MPI_Error_class(code) == code & 0x7f and
 * MPI_Error_string prints the stack ("FCNAME(line): message" per level, the
 * format of MPIR_Err_print_stack_string, errutil.c:1067-1160).  An
 * MPI_ERR_OTHER code wrapping a more specific one keeps the inner class
 * (errutil.c:896-905).  Messages use the texts of errnames.txt for the keys
 * this library raises; "%D" / "%O" print datatype / op names.
 */
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpir_op_types.h"

#define RING_SIZE 128           /* ERROR_SPECIFIC_INDEX_SIZE */
#define RING_SHIFT 19
#define SEQ_SHIFT 26
#define CLASS_MASK 0x7f
#define FATAL_MASK 0x80

typedef struct {
    int id;                     /* the code this entry was created for */
    int prev;                   /* lastcode */
    char location[64];
    char msg[257];
} ring_entry;

static ring_entry ring[RING_SIZE];
static unsigned ring_loc, ring_seq;
static pthread_mutex_t ring_lock = PTHREAD_MUTEX_INITIALIZER;

/* errnames.txt texts of the keys raised here (specific forms first) */
static const struct {
    const char *key, *text;
} msgs[] = {
    {"**mpi_reduce_local %p %p %d %D %O",
     "MPI_Reduce_local(inbuf=%p, inoutbuf=%p, count=%d, datatype=%D, op=%O) failed"},
    {"**mpi_reduce_local", "MPI_Reduce_local failed"},
    {"**opnull", "Null MPI_Op"},
    {"**opnotallowed", "MPI_Op operation is not allowed in this routine"},
    {"**opundefined %s", "MPI_Op %s operation not defined for this datatype"},
    {"**opundefined", "MPI_Op operation not defined for this datatype"},
    {"**permop", "Cannot free permanent MPI_Op"},
    {"**bufalias", "Buffers must not be aliased"},
    {"**buf_inplace %s", "buffer '%s' cannot be MPI_IN_PLACE"},
    {"**nomem %s", "Out of memory (unable to allocate a '%s')"},
    {"**other", "Other MPI error"},
};

static const char *lookup(const char *key)
{
    for (size_t i = 0; i < sizeof(msgs) / sizeof(msgs[0]); i++)
        if (!strcmp(msgs[i].key, key))
            return msgs[i].text;
    return key;
}

static const char *op_name(int op)
{
    static const char *names[15] = { "MPI_OP_NULL", "MPI_MAX", "MPI_MIN", "MPI_SUM", "MPI_PROD", "MPI_LAND",
        "MPI_BAND", "MPI_LOR", "MPI_BOR", "MPI_LXOR", "MPI_BXOR", "MPI_MINLOC", "MPI_MAXLOC",
        "MPI_REPLACE", "MPI_NO_OP"
    };
    if (op == MPI_OP_NULL)
        return "MPI_OP_NULL";
    if (((unsigned) op & 0xfffffff0u) == 0x58000000u && (op & 0xf) < 15)
        return names[op & 0xf];
    return NULL;
}

/* vsnprintf_mpi (errutil.c) subset: %p %d %i %x %s %L, %D datatype, %O op */
static void format(char *out, size_t n, const char *fmt, va_list ap)
{
    size_t o = 0;
    char tmp[64];
    for (const char *f = fmt; *f && o + 1 < n; f++) {
        const char *s = tmp;
        if (*f != '%' || !f[1]) {
            out[o++] = *f;
            continue;
        }
        switch (*++f) {
        case 'd':
        case 'i':
            snprintf(tmp, sizeof tmp, "%d", va_arg(ap, int));
            break;
        case 'x':
            snprintf(tmp, sizeof tmp, "%x", va_arg(ap, unsigned));
            break;
        case 'L':
            snprintf(tmp, sizeof tmp, "%lld", va_arg(ap, long long));
            break;
        case 'p':
            snprintf(tmp, sizeof tmp, "%p", va_arg(ap, void *));
            break;
        case 's':
            s = va_arg(ap, const char *);
            if (!s)
                s = "(null)";
            break;
        case 'D':{
                const int dt = va_arg(ap, int);
                const MPIR_Type_desc *d = MPIR_Type_lookup(dt);
                if (d)
                    s = d->name;
                else
                    snprintf(tmp, sizeof tmp, "dtype=0x%x", (unsigned) dt);
                break;
            }
        case 'O':{
                const int op = va_arg(ap, int);
                s = op_name(op);
                if (!s) {
                    snprintf(tmp, sizeof tmp, "op=0x%x", (unsigned) op);
                    s = tmp;
                }
                break;
            }
        case '%':
            s = "%";
            break;
        default:
            snprintf(tmp, sizeof tmp, "%%%c", *f);
        }
        while (*s && o + 1 < n)
            out[o++] = *s++;
    }
    out[o] = 0;
}

__attribute__ ((weak))
int MPIR_Err_create_code(int lastcode, int fatal, const char fcname[], int line, int error_class,
                         const char generic_msg[], const char specific_msg[], ...)
{
    va_list ap;
    int idx, code;
    if (error_class == MPI_ERR_OTHER && (lastcode & CLASS_MASK) > MPI_SUCCESS)
        error_class = lastcode & CLASS_MASK;
    pthread_mutex_lock(&ring_lock);
    idx = (int) (ring_loc++ % RING_SIZE);
    ring_seq = (ring_seq + 1) & 0xfu;
    code = (error_class & CLASS_MASK) | (idx << RING_SHIFT) | (int) (ring_seq << SEQ_SHIFT) |
        ((fatal || (lastcode & FATAL_MASK)) ? FATAL_MASK : 0);
    ring[idx].id = code;
    ring[idx].prev = lastcode;
    snprintf(ring[idx].location, sizeof ring[idx].location, "%s(%d)", fcname ? fcname : "(unknown)", line);
    va_start(ap, specific_msg);
    if (specific_msg)
        format(ring[idx].msg, sizeof ring[idx].msg, lookup(specific_msg), ap);
    else
        snprintf(ring[idx].msg, sizeof ring[idx].msg, "%s", lookup(generic_msg ? generic_msg : "**other"));
    va_end(ap);
    pthread_mutex_unlock(&ring_lock);
    return code;
}

/* the ring entry of a code, or -1 (a bare class, or an entry since overwritten) */
static int entry_of(int code)
{
    const int idx = (code >> RING_SHIFT) & (RING_SIZE - 1);
    if (code == MPI_SUCCESS || (code & ~(CLASS_MASK | FATAL_MASK)) == 0)
        return -1;
    return ring[idx].id == code ? idx : -1;
}

/* MPIR_Err_print_stack_string (errutil.c:1067-1160) */
static void print_stack(int code, char *str, size_t maxlen)
{
    size_t width = 0, o = 0;
    pthread_mutex_lock(&ring_lock);
    for (int c = code, e; (e = entry_of(c)) >= 0; c = ring[e].prev)
        if (strlen(ring[e].location) > width)
            width = strlen(ring[e].location);
    for (int c = code, e, depth = 0; (e = entry_of(c)) >= 0 && depth < RING_SIZE; c = ring[e].prev, depth++) {
        int n = snprintf(str + o, maxlen - o, "%s", ring[e].location);
        if (n < 0 || (size_t) n >= maxlen - o)
            break;
        o += (size_t) n;
        for (size_t k = strlen(ring[e].location); k < width && o + 1 < maxlen; k++)
            str[o++] = '.';
        n = snprintf(str + o, maxlen - o, ": %s\n", ring[e].msg);
        if (n < 0 || (size_t) n >= maxlen - o)
            break;
        o += (size_t) n;
    }
    str[o < maxlen ? o : maxlen - 1] = 0;
    pthread_mutex_unlock(&ring_lock);
}

static const char *class_string(int cls)
{
    switch (cls) {
    case MPI_SUCCESS:
        return "No MPI error";
    case MPI_ERR_BUFFER:
        return "Invalid buffer pointer";
    case MPI_ERR_COUNT:
        return "Invalid count";
    case MPI_ERR_TYPE:
        return "Invalid datatype";
    case 5:    /* MPI_ERR_COMM */
        return "Invalid communicator";
    case 7:    /* MPI_ERR_ROOT */
        return "Invalid root";
    case MPI_ERR_OP:
        return "Invalid MPI_Op";
    case MPI_ERR_ARG:
        return "Invalid argument";
    case 14:   /* MPI_ERR_TRUNCATE */
        return "Message truncated";
    case MPI_ERR_OTHER:
        return "Other MPI error";
    case MPI_ERR_INTERN:
        return "Internal MPI error!";
    case MPI_ERR_NO_MEM:
        return "Out of memory";
    default:
        return "Unknown error class";
    }
}

__attribute__ ((weak))
int MPI_Error_class(int errorcode, int *errorclass)
{
    *errorclass = errorcode & CLASS_MASK;       /* error_class.c:76 */
    return MPI_SUCCESS;
}

__attribute__ ((weak))
int MPI_Error_string(int errorcode, char *string, int *resultlen)
{
    int n = snprintf(string, MPI_MAX_ERROR_STRING, "%s", class_string(errorcode & CLASS_MASK));
    if (n > 0 && n < MPI_MAX_ERROR_STRING && entry_of(errorcode) >= 0) {
        int m = snprintf(string + n, (size_t) (MPI_MAX_ERROR_STRING - n), ", error stack:\n");
        if (m > 0 && n + m < MPI_MAX_ERROR_STRING) {
            print_stack(errorcode, string + n + m, (size_t) (MPI_MAX_ERROR_STRING - n - m));
            n = (int) strlen(string);
            if (n > 0 && string[n - 1] == '\n')
                string[--n] = 0;
        }
    }
    if (n >= MPI_MAX_ERROR_STRING)
        n = MPI_MAX_ERROR_STRING - 1;
    *resultlen = n;
    return MPI_SUCCESS;
}

/* MPIR_Err_return_comm (errutil.c:238-341) with comm_ptr NULL: the default
 * handler, COMM_WORLD's.  This library has no communicator objects, so the
 * handler is the one MPIX_Reduce_local_set_errhandler sets (fatal by default). */
__attribute__ ((weak))
int MPIR_Err_return_comm(void *comm_ptr, const char fcname[], int errcode)
{
    MPI_Errhandler h = MPI_ERRORS_ARE_FATAL;
    (void) comm_ptr;
    MPIX_Reduce_local_get_errhandler(&h);
    if (h == MPI_ERRORS_ARE_FATAL || (errcode & FATAL_MASK)) {
        char stack[MPI_MAX_ERROR_STRING];
        print_stack(errcode, stack, sizeof stack);
        fprintf(stderr, "Fatal error in %s: %s, error stack:\n%s", fcname, class_string(errcode & CLASS_MASK),
                stack[0] ? stack : "(no stack)\n");
        fflush(stderr);
        exit(1);
    }
    return errcode;
}
