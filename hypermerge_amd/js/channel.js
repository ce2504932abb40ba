'use strict'
// channel.js — the buffered push/subscribe channel that DocBackend exposes as `ready`
// and uses for its change queues.  Delivery contract of the reference's Queue
// (src/Queue.ts:1-77): before a subscriber exists, pushed items wait in FIFO order;
// subscribing delivers the backlog synchronously, and from then on `push` is the
// subscriber itself, so a push runs the subscriber inside the pusher's stack.
// unsubscribe() returns to buffering; once() takes exactly one item.

class Channel {
  constructor(label) {
    this.label = label || 'unknown'
    this.backlog = []
    this.sink = null
    this.buffer = (item) => { this.backlog.push(item) }
    this.push = this.buffer
  }

  get length() { return this.backlog.length }

  subscribe(sink) {
    if (this.sink) throw new Error(`${this.label}: only one subscriber at a time to a queue`)
    this.sink = sink
    // a sink may unsubscribe (or be replaced) while the backlog drains
    while (this.sink === sink) {
      if (this.backlog.length === 0) { this.push = sink; return }
      sink(this.backlog.shift())
    }
  }

  unsubscribe() {
    this.sink = null
    this.push = this.buffer
  }

  once(fn) {
    if (this.sink) return
    const one = (item) => { this.unsubscribe(); fn(item) }
    this.subscribe(one)
  }

  first() { return new Promise((resolve) => this.once(resolve)) }

  drain(fn) {
    // items pushed by fn are drained too
    for (let x = this.backlog.shift(); x !== undefined || this.backlog.length; x = this.backlog.shift()) {
      if (x !== undefined) fn(x)
    }
  }
}

module.exports = Channel
