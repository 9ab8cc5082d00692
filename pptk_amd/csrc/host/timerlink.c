/*
 * timerlink.c -- timer heap of include/timerlink.h: a skew heap (self-
 * adjusting meldable heap) on the timer_link parent/left/right links.  Add,
 * remove-any and modify are O(log n) amortized; the root is always the
 * earliest timer, which is all the reference's API promises
 * (timerlinkheap/timerlink.h).  Merges are iterative (top-down), so no
 * recursion depth grows with the heap.
 */
#include "timerlink.h"

/* Top-down skew merge of two heaps (either may be NULL); the result's
 * parent link is left for the caller.  At each step the smaller root keeps
 * its left subtree as its right one and takes, as its left, the merge of
 * its old right subtree with the other heap. */
static struct timer_link *merge(struct timer_link *a, struct timer_link *b)
{
  struct timer_link *root, *t;
  if (!a)
    return b;
  if (!b)
    return a;
  if (b->time64 < a->time64) {
    t = a;
    a = b;
    b = t;
  }
  root = a;
  for (;;) {
    struct timer_link *r = a->right;
    a->right = a->left;
    if (!r) {
      a->left = b;
      b->parent = a;
      break;
    }
    if (b->time64 < r->time64) {
      t = r;
      r = b;
      b = t;
    }
    a->left = r;
    r->parent = a;
    a = r;
  }
  return root;
}

void timer_linkheap_add(struct timer_linkheap *heap, struct timer_link *timer)
{
  timer->parent = timer->left = timer->right = NULL;
  heap->root = merge(heap->root, timer);
  heap->root->parent = NULL;
  heap->size++;
}

void timer_linkheap_remove(struct timer_linkheap *heap, struct timer_link *timer)
{
  struct timer_link *sub = merge(timer->left, timer->right);
  struct timer_link *p = timer->parent;
  if (sub)
    sub->parent = p;
  if (!p)
    heap->root = sub;
  else if (p->left == timer)
    p->left = sub;
  else
    p->right = sub;
  timer->parent = timer->left = timer->right = NULL;
  heap->size--;
}

void timer_linkheap_modify(struct timer_linkheap *heap, struct timer_link *timer)
{
  timer_linkheap_remove(heap, timer);
  timer_linkheap_add(heap, timer);
}

/* Walks the tree along the parent links (no stack: skew heaps can be
 * deep), checking every child's back link and heap order, and counts it. */
int timer_linkheap_verify(struct timer_linkheap *heap)
{
  const struct timer_link *x = heap->root, *prev = NULL;
  size_t n = 0;
  int ok = !x || !x->parent;
  while (x) {
    const struct timer_link *next;
    if (prev == x->parent) {            /* first visit: check, go left */
      n++;
      if ((x->left && (x->left->parent != x || x->left->time64 < x->time64)) ||
          (x->right && (x->right->parent != x || x->right->time64 < x->time64)))
        ok = 0;
      next = x->left ? x->left : x->right ? x->right : x->parent;
    } else if (prev == x->left && x->left) {   /* back from the left */
      next = x->right ? x->right : x->parent;
    } else {                            /* back from the right */
      next = x->parent;
    }
    prev = x;
    x = next;
  }
  return ok && n == heap->size;
}
